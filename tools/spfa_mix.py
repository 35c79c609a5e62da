"""The SPFA pop mix on the host (round 4): which share of the reference SPFA's pops (pyx:89-107) the
path kernel's asm fast loop (spfa_fast_pops) can take.  A pop is "common" when >= 3 queue entries
remain after it, none of its pushes is below the front's distance (no SLF swap, pyx:104-107), and it
does not lower the front's distance; the rest go to the C++ pop.  Replays the SPFA from each robot's
snapped position on its own cspace, BASELINE scenes.

    python tools/spfa_mix.py [--envs 6] [--config lifting_4-small_divider]

Test infrastructure only (the oracle's cspace and snap)."""
import argparse
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')]

S2 = np.float32(np.sqrt(2))
ONE = np.float32(1)
DIRS = [(0, -1), (0, 1), (-1, -1), (-1, 0), (-1, 1), (1, -1), (1, 0), (1, 1)]  # pyx:30
WTS = [ONE, ONE, S2, ONE, S2, S2, ONE, S2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=6)
    ap.add_argument('--config', default='lifting_4-small_divider')
    args = ap.parse_args()
    import oracle as O
    from simaps import synthetic
    kinds, pushes = Counter(), Counter()
    tot = 0
    for e in range(args.envs):
        sc = synthetic.make_scene(args.config, e)
        for a in range(len(sc['robots'])):
            ao = O.AgentOracle(sc, a)
            g = ao.cspace.astype(bool)
            H, W = g.shape
            s = ao.snap(sc['robots'][a]['position'])
            d = np.full(H * W, np.float32(2 * H * W), np.float32)
            inq = np.zeros(H * W, bool)
            q = [0] * (H * W * 8 + 2)
            head = tail = 0
            u0 = s[0] * W + s[1]
            d[u0] = 0
            tail += 1
            q[tail] = u0
            inq[u0] = True
            while head < tail:
                head += 1
                u = q[head]
                inq[u] = False
                ui, uj = divmod(u, W)
                left = tail - head
                F0 = q[head + 1] if left > 0 else -1
                dF0 = d[F0] if F0 >= 0 else None
                fm = sw = False
                npush = 0
                for (di, dj), w in zip(DIRS, WTS):
                    i, j = ui + di, uj + dj
                    if i < 0 or j < 0 or i >= H or j >= W or not g[i, j]:
                        continue
                    v = i * W + j
                    nd = np.float32(d[u] + w)
                    if nd < d[v]:
                        fm |= v == F0
                        d[v] = nd
                        if not inq[v]:
                            npush += 1
                            sw |= dF0 is not None and nd < dF0
                            tail += 1
                            q[tail] = v
                            inq[v] = True
                            if d[q[tail]] < d[q[head + 1]]:
                                q[tail], q[head + 1] = q[head + 1], q[tail]
                tot += 1
                pushes[min(npush, 3)] += 1
                kinds['small_queue' if left < 3 else ('front_lowered' if fm else ('swap' if sw else 'common'))] += 1
    print(json.dumps({'config': args.config, 'pops': tot, 'kinds': {k: v / tot for k, v in kinds.items()},
                      'pushes_per_pop': {str(k) + ('+' if k == 3 else ''): v / tot for k, v in sorted(pushes.items())}}))


if __name__ == '__main__':
    main()
