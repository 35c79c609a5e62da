"""Host model of get_state_kernel's SSSP sweep schedule ("SSSP sweeps"): how many
line steps the dirty-line marking spends, and how many a finer marking rule would spend.

    python tools/sweep_sim.py [--config lifting_4-small_divider] [--envs 16]

Per source, four directional sweeps (down / up / right / left) relax a line from the 3 cells of the
previous line (f32 distances, weights 1 and f32(sqrt 2), like shortest_paths.pyx:29-31).  Rounds
run the four sweeps on masks snapshotted at the round start (marks made during a round go to the
next one; the value updates within a round are applied in sweep order, a sequential stand-in for
the concurrent waves).  A sweep starts at its first dirty line and stops at the first 4 non-improving
lines past its last dirty line.  Two marking rules:

  current  (the kernel's): a lowered line is marked for the opposite direction; the lines (columns
           for the vertical sweeps) of its improving lanes are marked for both perpendicular ones;
  checked  a lowered cell marks only what an exact f32 relaxation check says it can improve: the
           opposite direction if it lowers a cell of the previous line (the sweep holds that line in
           registers), the perpendicular direction toward a same-line neighbour it lowers (DPP
           neighbour in the same step).  The other neighbours are the sweep's own next line.

Both reach the same fixpoint (checked against the oracle's SPFA here).  Prints per-direction line
steps for both rules and the kernel's stamp counts for comparison.  Test infrastructure only.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')]

S2 = np.float32(np.sqrt(2))
INF = np.float32(np.inf)


def relax_line(prev, cur, free_cur):
    """cur' = min(cur, prev[c-1] + s2, prev[c] + 1, prev[c+1] + s2) on free cells (f32)."""
    cand = prev + np.float32(1)
    d = prev + S2
    cand[1:] = np.minimum(cand[1:], d[:-1])
    cand[:-1] = np.minimum(cand[:-1], d[1:])
    new = np.where(free_cur, np.minimum(cur, cand), cur)
    return new


def simulate(free, src, rule):
    H, W = free.shape
    dist = np.full((H, W), INF, np.float32)
    dist[src] = 0
    # direction -> (axis, step); line index along the axis; masks are sets of line indices
    dirs = {'down': (0, 1), 'up': (0, -1), 'right': (1, 1), 'left': (1, -1)}
    opp = {'down': 'up', 'up': 'down', 'right': 'left', 'left': 'right'}
    masks = {'down': {src[0]}, 'up': {src[0]}, 'right': {src[1]}, 'left': {src[1]}}
    steps = {k: 0 for k in dirs}
    rounds = 0
    while any(masks.values()):
        rounds += 1
        snap = {k: set(v) for k, v in masks.items()}
        masks = {k: set() for k in dirs}
        for name, (axis, st) in dirs.items():
            m = snap[name]
            if not m:
                continue
            n = H if axis == 0 else W
            order = list(range(n)) if st > 0 else list(range(n - 1, -1, -1))
            pos = {l: i for i, l in enumerate(order)}
            first = min(pos[l] for l in m)
            last = max(pos[l] for l in m)
            quiet = 0
            for i in range(first, n - 1):
                k, k1 = order[i], order[i + 1]
                if axis == 0:
                    prev, cur, fr = dist[k], dist[k1], free[k1]
                else:
                    prev, cur, fr = dist[:, k], dist[:, k1], free[:, k1]
                new = relax_line(prev.copy(), cur.copy(), fr)
                steps[name] += 1
                imp = new < cur
                if axis == 0:
                    dist[k1] = new
                else:
                    dist[:, k1] = new
                if imp.any():
                    quiet = 0
                    idx = np.nonzero(imp)[0]
                    pa, pb = ('right', 'left') if axis == 0 else ('down', 'up')
                    if rule == 'current':
                        masks[opp[name]].add(k1)
                        for c in idx:
                            masks[pa].add(int(c))
                            masks[pb].add(int(c))
                    else:
                        # backward check: does line k1 lower any cell of line k?
                        back = relax_line(new.copy(), prev.copy(), free[k] if axis == 0 else free[:, k])
                        if (back < prev).any():
                            masks[opp[name]].add(k1)
                        # same-line checks: does cell c lower its neighbour c+1 (toward +) / c-1 (toward -)?
                        frl = fr
                        up = np.zeros_like(imp)
                        dn = np.zeros_like(imp)
                        up[:-1] = imp[:-1] & frl[1:] & (new[:-1] + np.float32(1) < new[1:])
                        dn[1:] = imp[1:] & frl[:-1] & (new[1:] + np.float32(1) < new[:-1])
                        for c in np.nonzero(up)[0]:
                            masks[pa].add(int(c))
                        for c in np.nonzero(dn)[0]:
                            masks[pb].add(int(c))
                else:
                    quiet += 1
                    if i >= last and quiet >= 4:
                        break
    return dist, steps, rounds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=16)
    args = ap.parse_args()
    import oracle
    from simaps import synthetic
    tot = {r: {} for r in ('current', 'checked')}
    rnds = {r: [] for r in tot}
    n = 0
    for e in range(args.envs):
        sc = synthetic.make_scene(args.config, e)
        for a in range(len(sc['robots'])):
            ao = oracle.AgentOracle(sc, a)
            srcs = [ao.snap(sc['robots'][a]['position'])]
            if sc['receptacle_position'] is not None:
                srcs.insert(0, ao.snap(sc['receptacle_position']))
            rows, cols = np.nonzero(ao.cspace)
            i0, i1, j0, j1 = rows.min(), rows.max() + 1, cols.min(), cols.max() + 1
            free = ao.cspace[i0:i1, j0:j1].astype(bool)
            for si, s in enumerate(srcs):
                ref = oracle.spfa_image(ao.cspace, s)[i0:i1, j0:j1]
                for rule in tot:
                    d, st, r = simulate(free, (s[0] - i0, s[1] - j0), rule)
                    d = np.where(np.isinf(d), np.float32(-1), d)
                    assert np.array_equal(np.where(free, d, 0), np.where(free, ref, 0)), (e, a, si, rule)
                    for k, v in st.items():
                        tot[rule].setdefault((si, k), []).append(v)
                    rnds[rule].append(r)
            n += 1
    out = {'config': args.config, 'agents': n, 'room': list(free.shape)}
    for rule in tot:
        out[rule] = {'source%d_%s' % k: float(np.median(v)) for k, v in sorted(tot[rule].items())}
        out[rule]['rounds_median'] = float(np.median(rnds[rule]))
        out[rule]['steps_total_median_per_source'] = float(np.median(
            [sum(tot[rule][(si, k)][i] for k in ('down', 'up', 'right', 'left'))
             for si in {k[0] for k in tot[rule]} for i in range(n)]))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
