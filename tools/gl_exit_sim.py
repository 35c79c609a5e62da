"""Large-window movement path early exit, modelled on the host (round 6): for random queries on a
500 x 500 grid (25 % obstacles, the bench's seed), the SPFA replay's total pops, the first pop after
which the target's parent chain holds its fixpoint distances (`exact`, checked every 64 pops, what
gl_path_kernel's incremental check sees), and the pop at which round 5's schedule -- a full chain
walk at doubling intervals 32, 96, 224, ... -- noticed it (None: never before the queue emptied).
Test infrastructure only (the oracle's SPFA image is the fixpoint).

    python tools/gl_exit_sim.py
"""
import sys, time
import numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'oracle')]
import oracle as O
S2 = np.float32(np.sqrt(2)); ONE = np.float32(1)
DIRS = [(0, -1), (0, 1), (-1, -1), (-1, 0), (-1, 1), (1, -1), (1, 0), (1, 1)]
WTS = [ONE, ONE, S2, ONE, S2, S2, ONE, S2]

def trace(grid, src, tgt, F):
    H, W = grid.shape
    INF = np.float32(np.inf)
    d = np.full(H * W, INF, np.float32); par = np.full(H * W, -1, np.int64); inq = np.zeros(H * W, bool)
    from collections import deque
    q = [0] * (H * W * 8 + 2); head = tail = 0
    s = src[0] * W + src[1]; t = tgt[0] * W + tgt[1]
    d[s] = 0; tail += 1; q[tail] = s; inq[s] = True
    pops = 0; exact = None; sched = None; lim, gap = 32, 64
    def chain_final():
        v = t
        if d[v] != F[v]: return False
        while v != s:
            v = par[v]
            if v < 0 or d[v] != F[v]: return False
        return True
    free = grid.ravel()
    while head < tail:
        head += 1; u = q[head]; inq[u] = False
        ui, uj = divmod(u, W)
        for (di, dj), w in zip(DIRS, WTS):
            i, j = ui + di, uj + dj
            if i < 0 or j < 0 or i >= H or j >= W or not free[i * W + j]: continue
            v = i * W + j
            nd = np.float32(d[u] + w)
            if nd < d[v]:
                par[v] = u; d[v] = nd
                if not inq[v]:
                    tail += 1; q[tail] = v; inq[v] = True
                    if d[q[tail]] < d[q[head + 1]]:
                        q[tail], q[head + 1] = q[head + 1], q[tail]
        pops += 1
        if exact is None and pops % 64 == 0 and chain_final(): exact = pops
        if sched is None and pops == lim:
            if chain_final(): sched = pops
            else:
                lim = pops + gap; gap = min(gap * 2, 1 << 20)
        if exact is not None and sched is not None: break
    return pops, exact, sched

rs = np.random.RandomState(505)
grid = (rs.random_sample((500, 500)) > 0.25).astype(np.uint8)
free = np.argwhere(grid != 0)
for k in range(4):
    src = tuple(free[rs.randint(len(free))]); tgt = tuple(free[rs.randint(len(free))])
    F = O.spfa_image(grid, src).ravel().astype(np.float32)
    F = np.where(F < 0, np.float32(np.inf), F)
    t0 = time.time()
    print(src, tgt, trace(grid.astype(bool), src, tgt, F), '%.0fs' % (time.time() - t0), flush=True)
