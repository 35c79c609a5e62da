"""The source hash baked into libsimaps.so at build time (simaps_source_hash, include/simaps.h).

One function computes it for both sides: the Makefile runs this file to pass the hash to hipcc
(-DSIMAPS_SOURCE_HASH), and simaps._lib recomputes it from the tree at load time and refuses a
library built from other sources -- a stale binary left over from before a kernel edit.  The
reference rebuilds its extension from its own source the same way (shortest_paths/setup.py:1-6).

Hashed: every `.hip` / `.h` / `.inc` file of spatial-intention-maps_amd/csrc and include/simaps.h,
in sorted relative-path order, each as `path NUL content NUL`.  Comments count: any edit of a
kernel source makes the library stale until it is rebuilt.
"""
import hashlib
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # spatial-intention-maps_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)


def source_files(pkg_root=PKG_ROOT, repo_root=None):
    """(relative path, absolute path) of every hashed source, in hash order."""
    repo_root = repo_root or os.path.dirname(pkg_root)
    csrc = os.path.join(pkg_root, 'csrc')
    files = [('csrc/' + f, os.path.join(csrc, f)) for f in os.listdir(csrc)
             if os.path.splitext(f)[1] in ('.hip', '.h', '.inc')]
    files.append(('include/simaps.h', os.path.join(repo_root, 'include', 'simaps.h')))
    return sorted(files)


def source_hash(pkg_root=PKG_ROOT, repo_root=None):
    """sha256 hex digest of the sources libsimaps.so is built from."""
    h = hashlib.sha256()
    for rel, path in source_files(pkg_root, repo_root):
        with open(path, 'rb') as f:
            h.update(rel.encode() + b'\0' + f.read() + b'\0')
    return h.hexdigest()


if __name__ == '__main__':
    print(source_hash())
