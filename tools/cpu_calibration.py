"""Calibrate the CPU baseline: the oracle ("port", what bench.py can time on
the GPU box) against the reference itself (envs.py OccupancyMap.update + Mapper.get_state with the
Cython GridGraph, imported as tests/golden/make_goldens.py does), on the same scenes, one process,
one thread each, in this dev container.  Writes profiles/r2_cpu_calibration.json.

    python tools/cpu_calibration.py [--envs 12] [--reps 3]

The unit is the same on both sides: one agent stack = the cspace / EDT / GridGraph work of
OccupancyMap.update for the agent's occupancy map WITHOUT the point scatter (the reference's
update() is called with an empty point cloud on a pre-filled occupancy map), then
Mapper.get_state().  Mapper construction and scene generation are outside the timed region.
The reference leg runs under the python3.9 oracle env (scipy 1.7.1 / skimage 0.18.3, SURVEY.md
8(c)) in a child process; the reference never leaves this container.
"""
import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
    os.environ[_v] = '1'
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
PY39 = '/opt/conda/bin/python3.9'
OUT = os.path.join(ROOT, 'profiles', 'r2_cpu_calibration.json')
CONFIGS = ['lifting_4-small_divider', 'lifting_1-small_empty', 'pushing_4-large_empty',
           'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty']


def leg_reference(config, envs):
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import numpy as np
    import make_goldens as MG
    from simaps import constants as K, synthetic
    ref_envs, _ = MG.import_reference()
    n, el = 0, 0.0
    for e in range(envs):
        scene = synthetic.make_scene(config, 90_000 + e)
        env = MG.build_env(ref_envs, scene)
        for a in range(len(scene['robots'])):
            m = ref_envs.Mapper(env, env.robots[a])
            m.global_overhead_map_without_robots[:] = scene['overhead'][a]
            om = m.global_occupancy_map
            om.occupancy_map[:] = scene['occupancy'][a]
            pts = np.zeros((1, 1, 3), np.float32)
            seg = np.full((1, 1), K.SEG_VALUES['floor'], np.float32)
            t0 = time.perf_counter()
            om.update(pts, seg, K.SEG_VALUES['obstacle'])
            m.get_state()
            el += time.perf_counter() - t0
            n += 1
    return n, el


def leg_port(config, envs):
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    from simaps import synthetic
    oracle.agent_state(synthetic.make_scene(config, 1), 0)
    n, el = 0, 0.0
    for e in range(envs):
        scene = synthetic.make_scene(config, 90_000 + e)
        for a in range(len(scene['robots'])):
            t0 = time.perf_counter()
            oracle.agent_state(scene, a)
            el += time.perf_counter() - t0
            n += 1
    return n, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--leg', choices=['reference', 'port'])
    ap.add_argument('--config', default=None)
    ap.add_argument('--envs', type=int, default=12)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    if args.leg:
        n, el = (leg_reference if args.leg == 'reference' else leg_port)(args.config, args.envs)
        print(json.dumps({'stacks': n, 'seconds': el}))
        return
    env = dict(os.environ)
    env.pop('PYTHONPATH', None)
    res = {'host': '', 'method': __doc__.split('\n\n')[0].replace('\n', ' ')}
    try:
        res['host'] = [l.split(':', 1)[1].strip() for l in open('/proc/cpuinfo') if l.startswith('model name')][0]
    except (OSError, IndexError):
        res['host'] = platform.processor()
    for cfg in ([args.config] if args.config else CONFIGS):
        rates = {'reference': [], 'port': []}
        for _ in range(args.reps):  # alternate the legs so drift hits both
            for leg in ('reference', 'port'):
                py = PY39 if leg == 'reference' else sys.executable
                o = subprocess.run([py, os.path.abspath(__file__), '--leg', leg, '--config', cfg, '--envs', str(args.envs)],
                                   env=env, capture_output=True, text=True, check=True)
                r = json.loads(o.stdout.strip().splitlines()[-1])
                rates[leg].append(r['stacks'] / r['seconds'])
        ref, port = statistics.median(rates['reference']), statistics.median(rates['port'])
        res[cfg] = {'reference_stacks_per_s': ref, 'port_stacks_per_s': port, 'port_over_reference': port / ref,
                    'runs': rates, 'stacks_per_run': args.envs * len(__import__('simaps.synthetic', fromlist=['x'])
                                                                   .make_scene(cfg, 0)['robots'])}
        print(cfg, json.dumps(res[cfg]), flush=True)
    json.dump(res, open(OUT, 'w'), indent=1)
    print('wrote', os.path.relpath(OUT, ROOT))


if __name__ == '__main__':
    main()
