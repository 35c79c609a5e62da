"""Parity fuzz of the SURVEY.md 8(f) rows on fresh seeds (GPU box): movement paths
(OccupancyMap.shortest_path, simaps_shortest_path) and reward lookups
(OccupancyMap.shortest_path_distance, simaps_sp_distance) of every agent's own map, against the CPU
oracle in a process pool.  A path mismatch is classified with the tests' approximate_polygon tie
check (tests/test_gpu_dropin.py::_dp_tie): at such a tie the reference's own pick is host-dependent.

    python tools/fuzz_rows.py [envs_per_config] [queries_per_agent] [procs] [--path-mode 0|1|2]
"""
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

CONFIGS = ['lifting_4-small_divider', 'pushing_4-large_empty', 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
           'lifting_4-large_doors', 'lifting_4-large_tunnels', 'lifting_4-large_rooms']
SEED0 = int(os.environ.get('SIMAPS_FUZZ_SEED0', '6000'))  # (--seed0 sets it for the spawned oracle workers too)


def queries(scene, e, a, Q):
    rs = np.random.RandomState(SEED0 + 31 * e + a)
    rl, rw = scene['room_length'], scene['room_width']
    src = np.array(scene['robots'][a]['position'][:2])
    tgt = np.stack([rs.uniform(-rl / 2 + 0.02, rl / 2 - 0.02, Q), rs.uniform(-rw / 2 + 0.02, rw / 2 - 0.02, Q)], -1)
    return src, tgt


def _oracle(job):
    import oracle as O
    from simaps import synthetic
    from test_gpu_dropin import _dp_tie
    cfg, e, a, Q, got_paths = job
    s = synthetic.make_scene(cfg, SEED0 + e, observe_all=True)
    ao = O.AgentOracle(s, a)
    src, tgt = queries(s, e, a, Q)
    dists = [ao.shortest_path_distance(src, t) for t in tgt]
    bad = ties = nontrivial = 0
    for t, got in zip(tgt, got_paths):
        want = np.array(ao.shortest_path(src, t), dtype=np.float64).reshape(-1, 2)
        nontrivial += len(want) > 2
        if not np.array_equal(np.array([p[:2] for p in got], dtype=np.float64).reshape(-1, 2), want):
            bad += 1
            ties += bool(_dp_tie(ao.cspace, ao.snap(src), ao.snap(t)))
    return dists, bad, ties, nontrivial


def main():
    argv = list(sys.argv[1:])
    mode = 0
    if '--path-mode' in argv:  # simaps_path_mode: 0 automatic, 1 compact, 2 early exit, 3 overlapped early exit
        k = argv.index('--path-mode')
        mode = int(argv[k + 1])
        del argv[k:k + 2]
    if '--seed0' in argv:  # first scene seed (default 6000): fresh seeds for a new fuzz run
        k = argv.index('--seed0')
        global SEED0
        SEED0 = int(argv[k + 1])
        os.environ['SIMAPS_FUZZ_SEED0'] = str(SEED0)
        del argv[k:k + 2]
    envs = int(argv[0]) if len(argv) > 0 else 16
    Q = int(argv[1]) if len(argv) > 1 else 4
    procs = int(argv[2]) if len(argv) > 2 else 16
    from simaps import _lib, batch, synthetic
    _lib.lib.simaps_path_mode(mode)
    tot = {'paths': 0, 'paths_with_detours': 0, 'path_mismatches': 0, 'at_ties': 0, 'lookups': 0, 'lookup_mismatches': 0}
    with get_context('spawn').Pool(procs) as pool:
        for cfg in CONFIGS:
            t0 = time.time()
            scenes = [synthetic.make_scene(cfg, SEED0 + e, observe_all=True) for e in range(envs)]
            b = batch.StateBatch(scenes)
            qs = [queries(scenes[e], e, a, Q) for e, a in b.agents]
            src = np.stack([q[0] for q in qs])
            tgt = np.stack([q[1] for q in qs])
            # one launch per query index: source k's q-th target, every agent at once
            paths = [b.shortest_paths(src, tgt[:, q]) for q in range(Q)]
            d = b.shortest_path_distances(src, tgt).cpu().numpy()
            jobs = [(cfg, e, a, Q, [paths[q][n] for q in range(Q)]) for n, (e, a) in enumerate(b.agents)]
            res = pool.map(_oracle, jobs, chunksize=2)
            r = {'config': cfg, 'paths': len(jobs) * Q, 'paths_with_detours': sum(x[3] for x in res),
                 'path_mismatches': sum(x[1] for x in res),
                 'at_ties': sum(x[2] for x in res), 'lookups': len(jobs) * Q,
                 'lookup_mismatches': int(sum(np.sum(np.array(x[0]) != d[n]) for n, x in enumerate(res)))}
            for k in tot:
                tot[k] += r[k]
            r['s'] = round(time.time() - t0, 1)
            print(json.dumps(r), flush=True)
    tot['seeds'] = [SEED0, SEED0 + envs - 1]
    tot['path_mode'] = mode
    print(json.dumps(tot), flush=True)


if __name__ == '__main__':
    main()
