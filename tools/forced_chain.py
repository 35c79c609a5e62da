"""VERDICT r3 item 2, measured on the host first: how often is a movement path's SPFA parent chain
FORCED by the fixpoint alone?  The SPFA's final parent of v lies in C(v) = {u : fl(F[u] + w_uv) ==
F[v]} (F = the f32 fixpoint); where |C(v)| = 1 along the whole chain from the target back to the
source, the path would follow from F without replaying the SPFA (shortest_paths.pyx:121-154).

    python tools/forced_chain.py [--envs 16]

For reference-like queries (OccupancyMap.shortest_path, envs.py:2478-2505: the robot's position to
a target in its local map (+-0.5 m, the action space) and to a target across the room) whose
straight line is blocked (the SPFA runs), prints the share of chains that are fully forced and the
share of forced chain vertices.  Test infrastructure only (the oracle's SPFA is the checker)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')]

S2 = np.float32(np.sqrt(2))
NB = [(-1, -1, S2), (-1, 0, np.float32(1)), (-1, 1, S2), (0, -1, np.float32(1)), (0, 1, np.float32(1)),
      (1, -1, S2), (1, 0, np.float32(1)), (1, 1, S2)]


def chain_stats(grid, src, tgt):
    import oracle as O
    H, W = grid.shape
    d, p = O.spfa(grid, src)
    d = d.reshape(H, W)
    u = src[0] * W + src[1]
    v = tgt[0] * W + tgt[1]
    if d[tgt] < 0:
        return None
    forced = total = 0
    while v != u:
        r, c = divmod(v, W)
        cands = 0
        for dr, dc, w in NB:
            rr, cc = r + dr, c + dc
            if 0 <= rr < H and 0 <= cc < W and grid[rr, cc] and d[rr, cc] >= 0 and np.float32(d[rr, cc] + w) == d[r, c]:
                cands += 1
        total += 1
        forced += cands == 1
        v = int(p[v])
    return forced, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=16)
    args = ap.parse_args()
    import oracle as O
    from simaps import synthetic
    out = {}
    for cfg in ('lifting_4-small_divider', 'lifting_4-large_doors', 'lifting_4-large_rooms'):
        for kind in ('local', 'across'):
            rs = np.random.RandomState(17)
            full = vert = tot = q = 0
            for e in range(args.envs):
                sc = synthetic.make_scene(cfg, 900 + e)
                for a in range(len(sc['robots'])):
                    ao = O.AgentOracle(sc, a)
                    x, y = sc['robots'][a]['position'][:2]
                    if kind == 'local':
                        t = (x + rs.uniform(-0.5, 0.5), y + rs.uniform(-0.5, 0.5))
                    else:
                        t = (-np.sign(x) * rs.uniform(0.05, sc['room_length'] / 2), rs.uniform(-sc['room_width'] / 2, sc['room_width'] / 2))
                    si, sj = O.position_to_pixel_indices(x, y, ao.shape)
                    ti, tj = O.position_to_pixel_indices(t[0], t[1], ao.shape)
                    rr, cc = O.line(si, sj, ti, tj)
                    if (1 - ao.cspace_thin[rr, cc]).sum() == 0:
                        continue  # straight line: no SPFA
                    st = chain_stats(ao.cspace, ao.snap((x, y)), ao.snap(t))
                    if st is None or st[1] == 0:
                        continue
                    q += 1
                    full += st[0] == st[1]
                    vert += st[0]
                    tot += st[1]
            out['%s/%s' % (cfg, kind)] = {'queries_with_spfa': q, 'fully_forced_chains': full,
                                         'share_fully_forced': full / max(q, 1), 'share_forced_vertices': vert / max(tot, 1),
                                         'chain_vertices': tot}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
