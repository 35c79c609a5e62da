"""Digest of one kernel's gfx950 assembly (hipcc --cuda-device-only -S output): line count and sha256 of
its body with labels renumbered, to check that a source edit elsewhere left a kernel's code unchanged.

    python tools/isa_digest.py file.s [kernel-substring ...]
"""
import hashlib
import re
import sys


def bodies(path, subs):
    s = open(path).read()
    for name in re.findall(r'^(_Z\w+):', s, re.M):
        if subs and not any(k in name for k in subs):
            continue
        i = s.index(name + ':')
        j = s.index('.Lfunc_end', i)
        body = s[i:j]
        # local labels / basic-block numbers shift with unrelated functions: normalise them
        body = re.sub(r'\.LBB\d+_\d+', '.LBB', body)
        body = re.sub(r'\s*;.*$', '', body, flags=re.M)  # comments (incl. trailing ones)
        yield name, len(body.splitlines()), hashlib.sha256(body.encode()).hexdigest()[:16]


if __name__ == '__main__':
    for n, lines, h in bodies(sys.argv[1], sys.argv[2:]):
        print('%-90s %7d %s' % (n[:90], lines, h))
