"""Path kernel early exit, modelled on the host (round 4): at which SPFA pop could a movement-path
query stop?  The SPFA may stop once every vertex on the target's parent chain holds its final
(fixpoint) distance -- then no parent on the chain can change (shortest_paths.pyx:97-99 updates a
parent only on a strict improvement).  For reference-like queries (tools/forced_chain.py's: the
robot's position to a target in its local map and to one across the room, straight line blocked)
this replays the reference SPFA (pyx:69-107) pop by pop and reports, per query, the total pops,
the first pop after which the chain is final (`exact`), and the pop at which the round-3 kernel's
check schedule notices it (`sched`: the target's distance every 32 pops, the chain walk at
doubling intervals 64, 128, ... once the target is final).

    python tools/exit_sim.py [--envs 8]

Test infrastructure only (the oracle's cspace, snap and SPFA are the checker)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')]

S2 = np.float32(np.sqrt(2))
ONE = np.float32(1)
DIRS = [(0, -1), (0, 1), (-1, -1), (-1, 0), (-1, 1), (1, -1), (1, 0), (1, 1)]  # pyx:30
WTS = [ONE, ONE, S2, ONE, S2, S2, ONE, S2]


def spfa_trace(grid, src, tgt, F, interval=32):
    """Replay pyx:69-107; returns (total pops, exact exit pop, scheduled exit pop)."""
    H, W = grid.shape
    INF = np.float32(2 * H * W)
    d = np.full(H * W, INF, np.float32)
    par = np.full(H * W, -1, np.int64)
    inq = np.zeros(H * W, bool)
    q = [0] * (H * W * 8 + 2)
    head = tail = 0
    s = src[0] * W + src[1]
    t = tgt[0] * W + tgt[1]
    d[s] = 0
    tail += 1
    q[tail] = s
    inq[s] = True
    pops = 0
    exact = sched = None
    lim, gap = interval, 64

    def chain_final():
        v = t
        if d[v] != F[v]:
            return False
        while v != s:
            v = par[v]
            if v < 0 or d[v] != F[v]:
                return False
        return True

    while head < tail:
        head += 1
        u = q[head]
        inq[u] = False
        ui, uj = divmod(u, W)
        for (di, dj), w in zip(DIRS, WTS):
            i, j = ui + di, uj + dj
            if i < 0 or j < 0 or i >= H or j >= W or not grid[i, j]:
                continue
            v = i * W + j
            nd = np.float32(d[u] + w)
            if nd < d[v]:
                par[v] = u
                d[v] = nd
                if not inq[v]:
                    tail += 1
                    q[tail] = v
                    inq[v] = True
                    if d[q[tail]] < d[q[head + 1]]:
                        q[tail], q[head + 1] = q[head + 1], q[tail]
        pops += 1
        if exact is None and chain_final():
            exact = pops
        if sched is None and pops == lim:
            lim = pops + interval
            if d[t] == F[t]:
                if chain_final():
                    sched = pops
                else:
                    lim = pops + gap
                    gap *= 2
    return pops, exact if exact is not None else pops, sched if sched is not None else pops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=8)
    ap.add_argument('--interval', type=int, default=32, help='pops between target checks (the kernel: 32)')
    args = ap.parse_args()
    import oracle as O
    from simaps import synthetic
    out = {}
    for cfg in ('lifting_4-small_divider', 'lifting_4-large_rooms'):
        for kind in ('local', 'across'):
            rs = np.random.RandomState(17)
            rows = []
            for e in range(args.envs):
                sc = synthetic.make_scene(cfg, 900 + e)
                for a in range(len(sc['robots'])):
                    ao = O.AgentOracle(sc, a)
                    x, y = sc['robots'][a]['position'][:2]
                    if kind == 'local':
                        tp = (x + rs.uniform(-0.5, 0.5), y + rs.uniform(-0.5, 0.5))
                    else:
                        tp = (-np.sign(x) * rs.uniform(0.05, sc['room_length'] / 2),
                              rs.uniform(-sc['room_width'] / 2, sc['room_width'] / 2))
                    si, sj = O.position_to_pixel_indices(x, y, ao.shape)
                    ti, tj = O.position_to_pixel_indices(tp[0], tp[1], ao.shape)
                    rr, cc = O.line(si, sj, ti, tj)
                    if (1 - ao.cspace_thin[rr, cc]).sum() == 0:
                        continue
                    src, tgt = ao.snap((x, y)), ao.snap(tp)
                    F, _ = O.spfa(ao.cspace, src)
                    F = np.asarray(F, np.float32).ravel()
                    if F[tgt[0] * ao.shape[1] + tgt[1]] < 0:
                        continue
                    F = np.where(F < 0, np.float32(2 * ao.shape[0] * ao.shape[1]), F)
                    rows.append(spfa_trace(ao.cspace.astype(bool), src, tgt, F, args.interval))
            r = np.array(rows, dtype=np.float64)
            out['%s/%s' % (cfg, kind)] = {
                'queries': len(rows), 'pops_median': float(np.median(r[:, 0])), 'pops_max': float(r[:, 0].max()),
                'exact_exit_over_pops_median': float(np.median(r[:, 1] / r[:, 0])),
                'sched_exit_over_pops_median': float(np.median(r[:, 2] / r[:, 0])),
                'exact_exit_pops_max': float(r[:, 1].max()), 'sched_exit_pops_max': float(r[:, 2].max())}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
