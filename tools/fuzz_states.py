"""Parity fuzz of get_state (GPU box): every agent of E fresh-seed envs per configuration, rendered
through the C ABI in one launch per configuration and compared bitwise with the CPU oracle (oracle
workers in a process pool; the nonspatial intention channels within 1e-7, like the GPU tests).
Seeds 5000+ are used by no test.  Prints one JSON line per configuration and a total.

    python tools/fuzz_states.py [envs_per_config] [procs] [--perturb] [--plain] [--mixed]

--plain renders and checks with the plain-dgemv rounding of scipy.ndimage.rotate's out_center
(rotate_plain.npz's host) instead of the FMA one; --perturb also leaves ~10 % of the robots in the
never-acted state (None waypoints / target / index, idle).  --mixed renders through the mixed-
configuration launch instead (MixedStateBatch): every configuration's envs, alternately in the
FMA and the plain rounding, interleaved env by env into launches of up to 8 configurations.
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

CONFIGS = ['lifting_1-small_empty', 'lifting_4-small_divider', 'pushing_4-large_empty', 'lifting_2_throwing_2-large_empty',
           'rescue_4-small_empty', 'lifting_4-small_divider-history', 'lifting_4-large_empty-line',
           'lifting_4-small_empty-circle', 'lifting_4-small_divider-spatial', 'lifting_4-large_empty-nonspatial',
           'lifting_2_pushing_2-large_empty-all', 'lifting_4-large_doors', 'lifting_4-large_tunnels',
           'lifting_4-large_rooms', 'lifting_2_throwing_2-large_doors', 'lifting_4-large_rooms-history']
SEED0 = int(os.environ.get('SIMAPS_FUZZ_SEED0', '5000'))  # (inherited by the spawned oracle workers)


def perturbed_scene(cfg, e, perturb, rounding='fma'):
    s = _perturbed_scene(cfg, e, perturb)
    s['rotate_rounding'] = rounding
    return s


def _perturbed_scene(cfg, e, perturb):
    """make_scene(cfg, SEED0 + e); with perturb, robots anywhere in the room but 2 cm from its edge
    (next to walls, on dividers: the snap slow path), headings half the time on exact multiples of
    45 deg (+-pi, -0.0 included), positions half the time on pixel corners, random idle flags, and
    one shortest_path_map_scale per configuration from {-0.5, 0, 0.25, 3}."""
    from simaps import synthetic
    s = synthetic.make_scene(cfg, SEED0 + e)
    if not perturb:
        return s
    rs = np.random.RandomState(SEED0 + 7919 * e + 1)
    rl, rw, H, W = s['room_length'], s['room_width'], s['H'], s['W']
    for r in s['robots']:
        x, y = rs.uniform(-rl / 2 + 0.02, rl / 2 - 0.02), rs.uniform(-rw / 2 + 0.02, rw / 2 - 0.02)
        if rs.rand() < 0.5:
            x, y = (np.floor(W / 2 + x * 96) - W / 2) / 96.0, (H / 2 - np.floor(H / 2 - y * 96)) / 96.0
        r['position'] = (float(x), float(y), 0)
        r['waypoint_positions'] = [r['position']] + list(r['waypoint_positions'][1:])
        r['heading'] = float(rs.choice([-np.pi, np.pi, -0.0, 0.0, np.pi / 4, -3 * np.pi / 4, np.pi / 2])
                             if rs.rand() < 0.5 else rs.uniform(-np.pi, np.pi))
        r['idle'] = bool(rs.rand() < 0.25)
        if rs.rand() < 0.1:  # never acted (Robot.__init__ / reset state)
            r.update(idle=True, waypoint_positions=None, waypoint_index=None, target_ee=None)
    scale = [-0.5, 0.0, 0.25, 3.0][sum(map(ord, cfg)) % 4]
    s['flags'] = dict(s['flags'], shortest_path_map_scale=scale)
    return s


def _oracle(job):
    import oracle as O
    cfg, e, a, perturb, rounding = job
    return O.agent_state(perturbed_scene(cfg, e, perturb, rounding), a)


def _matches(got, ref, flags, nr):
    from test_gpu_parity import _nonspatial_slice
    ns = _nonspatial_slice(flags, nr)
    if ns is None:
        return np.array_equal(got.view(np.int32), ref.view(np.int32))
    m = np.ones(got.shape[-1], bool)
    m[ns] = False
    return (np.array_equal(np.ascontiguousarray(got[..., m]).view(np.int32), np.ascontiguousarray(ref[..., m]).view(np.int32))
            and np.abs(got[..., ns] - ref[..., ns]).max() <= 1e-7)


def main_mixed(envs, procs, perturb):
    import torch
    from simaps import _lib, batch
    jobs = [(cfg, e, 'plain' if e % 2 else 'fma') for e in range(envs) for cfg in CONFIGS]  # interleaved
    launches, cur, keys = [], [], set()
    for cfg, e, r in jobs:
        s = perturbed_scene(cfg, e, perturb, r)
        k = batch.mixed_key(s)
        if k not in keys and len(keys) == _lib.MAX_MIXED:
            launches.append(cur)
            cur, keys = [], set()
        keys.add(k)
        cur.append(((cfg, e, r), s))
    if cur:
        launches.append(cur)
    total = bad = 0
    with get_context('spawn').Pool(procs) as pool:
        for li, launch in enumerate(launches):
            t0 = time.time()
            scenes = [s for _, s in launch]
            mb = batch.MixedStateBatch(scenes, layout='hwc')
            views = [v.cpu().numpy() for v in mb.states(mb.render())]
            torch.cuda.synchronize()
            _lib.check_faults()
            refs = pool.map(_oracle, [launch[e][0][:2] + (a, perturb, launch[e][0][2]) for e, a in mb.agents], chunksize=4)
            nb = sum(not _matches(views[n], refs[n], scenes[e]['flags'], len(scenes[e]['robots']))
                     for n, (e, a) in enumerate(mb.agents))
            assert len(mb.agents) < 2 or not np.array_equal(views[0].view(np.int32), refs[1].view(np.int32)), \
                'checker is vacuous'
            total += mb.N
            bad += nb
            print(json.dumps({'launch': li, 'configurations': len(mb.plan['cfgs']), 'envs': len(scenes), 'stacks': mb.N,
                              'mismatches': nb, 's': round(time.time() - t0, 1), 'perturbed': perturb}), flush=True)
    print(json.dumps({'mixed': True, 'launches': len(launches), 'total_stacks': total, 'mismatches': bad,
                      'seeds': [SEED0, SEED0 + envs - 1], 'perturbed': perturb, 'rotate_rounding': 'fma + plain'}), flush=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    if '--mixed' in sys.argv:
        return main_mixed(int(args[0]) if args else 16, int(args[1]) if len(args) > 1 else 16, '--perturb' in sys.argv)
    perturb = '--perturb' in sys.argv
    rounding = 'plain' if '--plain' in sys.argv else 'fma'
    envs = int(args[0]) if len(args) > 0 else 16
    procs = int(args[1]) if len(args) > 1 else 16
    import torch
    from simaps import batch, synthetic
    from test_gpu_parity import _nonspatial_slice
    total = bad = 0
    with get_context('spawn').Pool(procs) as pool:
        for cfg in CONFIGS:
            t0 = time.time()
            scenes = [perturbed_scene(cfg, e, perturb, rounding) for e in range(envs)]
            b = batch.StateBatch(scenes)
            st = b.as_hwc(b.render()).cpu().numpy()
            torch.cuda.synchronize()
            refs = pool.map(_oracle, [(cfg, e, a, perturb, rounding) for e, a in b.agents], chunksize=4)
            nb = 0
            for n, (e, a) in enumerate(b.agents):
                ns = _nonspatial_slice(scenes[e]['flags'], len(scenes[e]['robots']))
                got, ref = st[n], refs[n]
                if ns is None:
                    ok = np.array_equal(got.view(np.int32), ref.view(np.int32))
                else:
                    m = np.ones(got.shape[-1], bool)
                    m[ns] = False
                    ok = (np.array_equal(np.ascontiguousarray(got[..., m]).view(np.int32),
                                         np.ascontiguousarray(ref[..., m]).view(np.int32))
                          and np.abs(got[..., ns] - ref[..., ns]).max() <= 1e-7)
                nb += not ok
            # negative control: the checker must see a difference between two different agents
            control = len(b.agents) < 2 or not np.array_equal(st[0].view(np.int32), refs[1].view(np.int32))
            assert control, 'checker is vacuous'
            total += len(b.agents)
            bad += nb
            print(json.dumps({'config': cfg, 'stacks': len(b.agents), 'mismatches': nb, 's': round(time.time() - t0, 1),
                              'perturbed': perturb, 'rotate_rounding': rounding}), flush=True)
    print(json.dumps({'total_stacks': total, 'mismatches': bad, 'seeds': [SEED0, SEED0 + envs - 1], 'perturbed': perturb,
                      'rotate_rounding': rounding}),
          flush=True)


if __name__ == '__main__':
    main()
