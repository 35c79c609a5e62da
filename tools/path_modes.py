"""The opt-in fixpoint-parent path modes (simaps_path_mode 4 / 5) against the
exact SPFA replay (mode 0): agreement and launch time, GPU box.

Mode 4 / 5 run no SPFA: after the directional sweeps reach the f32 fixpoint D, the target's chain is
walked on D itself (parent of v = a neighbour u with fl(D(u) + w) == D(v); ties: smallest D(u), then
pyx:30 edge order (4), or edge order alone (5)), then approximate_polygon and the line-of-sight
pruning unchanged.  SURVEY.md 8(f) row 1 allows this looser parity: the same waypoints within
shortest_paths/demo.py:46-48's atol=2 (pixels), or an equal path length.

Reported, per mode:
  * the fuzz of tools/fuzz_rows.py (7 configurations x ENVS envs x 4 agents x 4 targets, fresh seeds):
    paths identical to mode 0's (which equal the reference's but at approximate_polygon float ties,
    DESIGN.md section 3), paths within atol 2 px on every waypoint (same waypoint count), paths with an
    equal waypoint-polyline length (|d| <= 1e-9 m), and the worst length difference;
  * the reference's own fixtures: paths.npz / maze_paths.npz (OccupancyMap.shortest_path) and
    grid_paths.npz (GridGraph.shortest_path): identical, within atol 2;
  * launch ms of 64 / 256 paths (local-map and across-room targets), HIP events, per mode.

    python tools/path_modes.py [--seed0 S] [--envs E]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tools')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

MODES = {0: 'exact', 4: 'fixpoint_min', 5: 'fixpoint_edge'}
PPM = 96.0


def _arg(name, default):
    if name in sys.argv:
        return type(default)(sys.argv[sys.argv.index(name) + 1])
    return default


def _polyline_len(p):
    p = np.asarray(p, dtype=np.float64).reshape(-1, 2)
    return float(np.sum(np.hypot(*np.diff(p, axis=0).T))) if len(p) > 1 else 0.0


def compare(ref, got, atol):
    """ref / got: lists of waypoint lists -> counts (identical, within atol, equal length) and the
    worst polyline length difference."""
    same = close = eqlen = 0
    worst = 0.0
    for a, b in zip(ref, got):
        a = np.asarray([q[:2] for q in a], dtype=np.float64).reshape(-1, 2)
        b = np.asarray([q[:2] for q in b], dtype=np.float64).reshape(-1, 2)
        same += bool(a.shape == b.shape and np.array_equal(a, b))
        close += bool(a.shape == b.shape and np.allclose(a, b, rtol=0.0, atol=atol))
        d = abs(_polyline_len(a) - _polyline_len(b))
        eqlen += d <= 1e-9
        worst = max(worst, d)
    return {'n': len(ref), 'identical': same, 'within_atol2': close, 'equal_length': eqlen, 'max_len_diff': worst}


def _add(tot, r):
    for k in ('n', 'identical', 'within_atol2', 'equal_length'):
        tot[k] = tot.get(k, 0) + r[k]
    tot['max_len_diff'] = max(tot.get('max_len_diff', 0.0), r['max_len_diff'])


def fuzz(envs, seed0):
    import fuzz_rows
    from simaps import _lib, batch, synthetic
    fuzz_rows.SEED0 = seed0
    out = {m: {} for m in MODES if m}
    for cfg in fuzz_rows.CONFIGS:
        t0 = time.time()
        scenes = [synthetic.make_scene(cfg, seed0 + e, observe_all=True) for e in range(envs)]
        b = batch.StateBatch(scenes)
        qs = [fuzz_rows.queries(scenes[e], e, a, 4) for e, a in b.agents]
        src = np.stack([q[0] for q in qs])
        tgt = np.stack([q[1] for q in qs])
        paths = {}
        for m in MODES:
            prev = _lib.lib.simaps_path_mode(m)
            paths[m] = [p for q in range(4) for p in b.shortest_paths(src, tgt[:, q])]
            _lib.lib.simaps_path_mode(prev)
        detours = sum(len(p) > 2 for p in paths[0])
        for m in out:
            r = compare(paths[0], paths[m], 2.0 / PPM + 1e-12)
            r.update(config=cfg, mode=MODES[m], detours=detours, s=round(time.time() - t0, 1))
            print(json.dumps(dict(r, kind='fuzz_vs_exact')), flush=True)
            _add(out[m], r)
    for m, r in out.items():
        r.update(kind='fuzz_vs_exact_total', mode=MODES[m], seeds=[seed0, seed0 + envs - 1])
        print(json.dumps(r), flush=True)
    return out


def fixtures():
    """The reference's own path goldens through every mode."""
    import goldens as G
    from simaps import _lib, batch, synthetic, vector_env

    def occ_groups(z, skip):
        groups = {}
        for k in z.files:
            if not k.endswith('_path') or skip(k):
                continue
            key = k[:-len('_path')]
            head, q = key.rsplit('_q', 1)
            cfg, rest = head.rsplit('_e', 1)
            e, a = (int(x) for x in rest.split('_a'))
            groups.setdefault(cfg, []).append((e, a, key))
        return groups

    res = []
    for m in MODES:
        prev = _lib.lib.simaps_path_mode(m)
        for name, seed, obs_all, skip in (('paths.npz', 60, False, lambda k: k.startswith('demo')),
                                          ('maze_paths.npz', 70, True, lambda k: k == 'longest_path')):
            z = G.load(name)
            ref, got = [], []
            for cfg, items in occ_groups(z, skip).items():
                scenes = [synthetic.make_scene(cfg, seed + e, observe_all=obs_all) for e in range(3)]
                b = batch.StateBatch(scenes)
                slots = [b.agents.index((e, a)) for e, a, _ in items]
                got += b.shortest_paths(np.stack([z[k + '_src'] for _, _, k in items]),
                                        np.stack([z[k + '_tgt'] for _, _, k in items]), slots=slots)
                ref += [z[k + '_path'] for _, _, k in items]
            res.append(dict(compare(ref, got, 2.0 / PPM + 1e-12), fixture=name, mode=MODES[m],
                            detours=sum(len(r) > 2 for r in ref)))
        z = G.load('grid_paths.npz')
        demo = G.load('sssp.npz')['demo_cspace']
        keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))
        ref = [z[k + '_path'] for k in keys]
        got = vector_env.GridGraph(demo).shortest_paths([(tuple(z[k + '_src']), tuple(z[k + '_tgt'])) for k in keys])
        s0 = G.load('paths.npz')
        ref += [s0['demo_%d_path' % q] for q in range(3)]
        got += vector_env.GridGraph(demo).shortest_paths([(tuple(s0['demo_%d_src' % q]), tuple(s0['demo_%d_tgt' % q]))
                                                          for q in range(3)])
        g_m = 0
        while 'rand_%d_grid' % g_m in z.files:
            gg = vector_env.GridGraph(z['rand_%d_grid' % g_m])
            pairs = [(tuple(z['rand_%d_%d_src' % (g_m, k)]), tuple(z['rand_%d_%d_tgt' % (g_m, k)])) for k in range(6)]
            got += gg.shortest_paths(pairs)
            ref += [z['rand_%d_%d_path' % (g_m, k)] for k in range(6)]
            g_m += 1
        res.append(dict(compare([np.asarray(r, float) for r in ref], [np.asarray(g, float) for g in got], 2.0),
                        fixture='grid_paths.npz', mode=MODES[m], detours=sum(len(r) > 2 for r in ref)))
        _lib.lib.simaps_path_mode(prev)
    for r in res:
        print(json.dumps(dict(r, kind='reference_fixture')), flush=True)
    return res


def timing():
    import path_bench
    out = []
    for cfg in ('lifting_4-small_divider', 'pushing_4-large_empty'):
        for targets in ('local', 'across'):
            for envs in (16, 64):
                for m in MODES:
                    out.append(path_bench.case(cfg, envs, 20, m, targets))  # (prints its own line)
    return out


def main():
    from simaps import _lib
    _lib.lib.simaps_fault_status(1)
    if '--no-timing' not in sys.argv:
        timing()
    fixtures()
    if '--no-fuzz' not in sys.argv:
        fuzz(_arg('--envs', 256), _arg('--seed0', 50000))
    _lib.check_faults()


if __name__ == '__main__':
    main()
