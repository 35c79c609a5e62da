"""Throughput of the SURVEY.md 8(f) rows built so far, GPU vs the CPU oracle (1 core):

  sp_distance    OccupancyMap.shortest_path_distance (reward lookups): queries/s
  shortest_path  OccupancyMap.shortest_path (movement paths): paths/s
  ingest         Robot.update_map minus the simulator (camera frame -> overhead / occupancy maps): frames/s
  distance_to_receptacle  the reward lookups from the receptacle, cold and from the render's cache
  env_step       (--env-step) the device time of one reference VectorEnv.step: paths, ingest, get_state
  mixed          (--mixed) one launch over envs of the BASELINE configurations together
                 (simaps_get_state_mixed) vs one launch per configuration back to back
  gridgraph_large (--gridgraph-large) GridGraph on a 500 x 500 grid (beyond the LDS window: the
                 global-memory kernels of csrc/grid_large.h): images and paths, 1 and 64 per call

    python tools/bench_extra.py [--config lifting_4-small_divider] [--envs 64] [--queries 8]

Prints one JSON line per row.  Inputs resident in HBM; timing with torch.cuda events around K
launches after warm-up.  The CPU leg times the oracle (the checker) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from simaps import batch, synthetic  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=64)
    ap.add_argument('--queries', type=int, default=8, help='reward-lookup targets per agent')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--cpu-budget', type=float, default=8.0)
    args = ap.parse_args()
    import oracle
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes)
    rs = np.random.RandomState(0)
    s0 = scenes[0]
    rl, rw = s0['room_length'], s0['room_width']
    N, Q = b.N, args.queries
    rec = s0['receptacle_position']
    src = np.array([rec[:2] if rec is not None else scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    tgt = np.stack([rs.uniform(-rl / 2, rl / 2, (N, Q)), rs.uniform(-rw / 2, rw / 2, (N, Q))], -1)
    src_d = torch.as_tensor(src).cuda()
    tgt_d = torch.as_tensor(tgt).cuda()
    dt = timed(lambda: b.shortest_path_distances(src_d, tgt_d), args.steps, 3)
    # CPU oracle on a bounded sample
    n, el = 0, 0.0
    for (e, a) in b.agents:
        t0 = time.perf_counter()
        ao = oracle.AgentOracle(scenes[e], a)
        k = b.agents.index((e, a))
        for q in range(Q):
            ao.shortest_path_distance(src[k], tgt[k, q])
        el += time.perf_counter() - t0
        n += Q
        if el > args.cpu_budget:
            break
    print(json.dumps({'row': 'sp_distance', 'config': args.config, 'agents': N, 'queries_per_agent': Q,
                      'gpu_queries_per_s': N * Q / dt, 'gpu_ms_per_launch': dt * 1e3,
                      'cpu_oracle_queries_per_s': n / el, 'cpu_cores': 1,
                      'cpu_sample': '%d queries incl. each agent\'s cspace / EDT / SPFA' % n}), flush=True)
    if rec is not None:
        # reward lookups from the receptacle (Mapper.distance_to_receptacle): cold = the full SSSP per
        # call (no cache); cached = the arrays the last render left (simaps_sp_lookup), as the
        # reference's GridGraph cache answers between two map updates
        cold = timed(lambda: b.receptacle_distances(tgt_d, cache=False), args.steps, 3)
        b.enable_receptacle_cache()
        b.render()
        cached = timed(lambda: b.receptacle_distances(tgt_d), args.steps, 3)
        assert (b._rec_ver == b._map_ver).all()
        got_c = b.receptacle_distances(tgt_d).cpu().numpy()
        got_f = b.receptacle_distances(tgt_d, cache=False).cpu().numpy()
        print(json.dumps({'row': 'distance_to_receptacle', 'config': args.config, 'agents': N, 'queries_per_agent': Q,
                          'cold_ms_per_call': cold * 1e3, 'cached_ms_per_call': cached * 1e3,
                          'cold_queries_per_s': N * Q / cold, 'cached_queries_per_s': N * Q / cached,
                          'cached_equals_cold': bool(np.array_equal(got_c, got_f)),
                          'note': 'StateBatch.receptacle_distances per call incl. host side; cached: every slot '
                                  'rendered since its last map change (simaps_sp_lookup), cold: cache=False '
                                  '(cspace + snap + SSSP per agent, simaps_sp_distance)'}), flush=True)

    # movement paths: robot position -> random target (half across x = 0)
    psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    ptgt = np.stack([rs.uniform(0.05, rl / 2, N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, N)], -1)
    dt = timed(lambda: b.shortest_paths(psrc, ptgt), max(3, args.steps // 4), 1)
    n, el = 0, 0.0
    for k, (e, a) in enumerate(b.agents):
        t0 = time.perf_counter()
        oracle.AgentOracle(scenes[e], a).shortest_path(psrc[k], ptgt[k])
        el += time.perf_counter() - t0
        n += 1
        if el > args.cpu_budget:
            break
    print(json.dumps({'row': 'shortest_path', 'config': args.config, 'paths_per_launch': N,
                      'gpu_paths_per_s': N / dt, 'gpu_ms_per_launch_incl_d2h': dt * 1e3,
                      'cpu_oracle_paths_per_s': n / el, 'cpu_cores': 1,
                      'cpu_sample': '%d paths incl. each agent\'s cspace / EDT / SPFA' % n}), flush=True)


def bench_dropin_step(args):
    """The drop-in's host + device cost of one observation step: VectorEnvObservations.update(new
    scene descriptors) + get_state() (device tensors, every robot), synchronised -- what a training
    loop pays per step beside its simulator (the bench line times the kernel alone)."""
    from simaps import vector_env
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    arrays = batch.descriptor_arrays(scenes)
    n = sum(len(s['robots']) for s in scenes)
    for mode in ('scenes', 'arrays', 'arrays+ring'):
        obs = vector_env.VectorEnvObservations(scenes, layout='chw', reuse_outputs=2 if mode == 'arrays+ring' else 0)
        if mode == 'scenes':
            upd = lambda: obs.update(scenes=scenes)  # noqa: E731
        else:
            upd = lambda: obs.update_arrays(**arrays)  # noqa: E731

        def step():
            upd()
            obs.get_state()
            torch.cuda.synchronize()
        for _ in range(5):
            step()
        ts, tu, tg = [], [], []
        for _ in range(max(args.steps, 300)):  # per-step times: the median resists the shared host's noise
            t0 = time.perf_counter()
            upd()
            t1 = time.perf_counter()
            obs.get_state()
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            ts.append(t3 - t0)
            tu.append(t1 - t0)
            tg.append(t2 - t1)
        dt = float(np.median(ts))
        print(json.dumps({'row': 'dropin_step', 'update': mode, 'config': args.config, 'stacks_per_step': n,
                          'ms_per_step': dt * 1e3, 'ms_per_step_mean': float(np.mean(ts)) * 1e3,
                          'host_update_ms': float(np.median(tu)) * 1e3, 'host_get_state_ms': float(np.median(tg)) * 1e3,
                          'stacks_per_s_end_to_end': n / dt,
                          'note': 'update(%s) + get_state() + synchronize, host packing and uploads included; '
                                  'median of %d steps' % (mode, len(ts))}),
              flush=True)


def bench_env_step(args):
    """the device work of one reference VectorEnv.step (envs.py:230-320) at
    BASELINE configs[1] (64 envs x 4 lifting robots), for E awaiting robots (default one per env, the
    steady state; --all: every robot, the first step): movement paths for the new actions
    (store_new_action -> Mapper.shortest_path, envs.py:234 -> 875-876; targets in the robot's local
    map, the action space), the awaiting robots' update_map (envs.py:277-280: a forward camera frame
    each) and their get_state render (envs.py:304, 322-323).  Each launch's device time by HIP
    events (K back-to-back launches of that part alone) and the three together, in step order, one
    stream.  Run it under rocprofv3 --kernel-trace --stats for the per-kernel split."""
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes)
    A = len(scenes[0]['robots'])
    slots = list(range(b.N)) if args.all else [e * A + (e % A) for e in range(args.envs)]
    n = len(slots)
    rs = np.random.RandomState(4)
    psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in (b.agents[k] for k in slots)])
    ptgt = psrc + rs.uniform(-0.5, 0.5, psrc.shape)   # inside the robot's local map
    src_d, tgt_d = torch.as_tensor(psrc).cuda(), torch.as_tensor(ptgt).cuda()
    frames = [synthetic.camera_images(scenes[e], a, 'forward', seed=k) for k, (e, a) in enumerate(b.agents[k] for k in slots)]
    dep = torch.as_tensor(np.stack([f[0] for f in frames])).cuda()
    seg = torch.as_tensor(np.stack([f[1] for f in frames]).astype(np.int32)).cuda()
    prep = b.prepare_ingest(dep, seg, camera='forward', slots=slots)
    out = b.alloc_state(n)
    s = torch.cuda.current_stream()
    parts = {'paths': lambda: b.launch_shortest_paths(src_d, tgt_d, slots=slots),
             'ingest': lambda: b.launch_ingest(prep),
             'get_state': lambda: b.render(out, slots=slots)}
    parts['step'] = lambda: [f() for f in (parts['paths'], parts['ingest'], parts['get_state'])]
    res = {}
    K = max(args.steps, 20)
    for name, f in parts.items():
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        res[name + '_us'] = e0.elapsed_time(e1) / K * 1e3
    print(json.dumps(dict({'row': 'env_step', 'config': args.config, 'awaiting_robots': n,
                           'note': 'device time per reference step (HIP events, %d launches each): movement paths '
                                   '(automatic path mode: the overlapped early-exit kernel at this size, local-map targets), forward-camera ingest, get_state of the '
                                   'awaiting robots; step = the three in order on one stream' % K}, **res)),
          flush=True)


def bench_remap(args):
    """The periodic re-map of one moving robot (RobotController.step -> update_map every 200
    simulation steps, envs.py:1401-1403): a single-frame simaps_ingest, end to end (host prep +
    upload + launch + synchronize, frame already on the device) and the two kernels alone."""
    from simaps import vector_env
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    obs = vector_env.VectorEnvObservations(scenes, layout='chw')
    db, raw = synthetic.camera_images(scenes[3], 2, 'forward', seed=1)
    dep, seg = torch.as_tensor(db[None]).cuda(), torch.as_tensor(raw[None]).cuda()

    def step():
        obs.update_map([(3, 2)], dep, seg)
        torch.cuda.synchronize()
    for _ in range(5):
        step()
    ts = []
    for _ in range(300):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    prep = obs.batch.prepare_ingest(dep, seg, camera='forward', slots=[obs.slot[(3, 2)]])
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(100):
        obs.batch.launch_ingest(prep)
    e1.record(s)
    torch.cuda.synchronize()
    print(json.dumps({'row': 'remap_one_robot', 'config': args.config, 'frames_per_launch': 1,
                      'ms_end_to_end': float(np.median(ts)) * 1e3, 'kernel_ms': e0.elapsed_time(e1) / 100,
                      'note': 'update_map([(env, robot)], frame) + synchronize, median of 300; kernels: HIP events '
                              'over 100 back-to-back launches'}), flush=True)


def bench_ingest(args):
    """Ingest row: the two kernels alone (HIP events on the launch stream around K launches of the
    device half, inputs resident) and end to end (host packing + upload + launch), with an HBM
    roofline: algorithmic bytes per frame = 8 B per camera pixel (depth f32 + seg i32 read once)
    + 5 B per map pixel (the overhead f32 / occupancy u8 maps it may rewrite)."""
    import oracle
    from simaps import camera
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes)
    kind = 'forward'
    frames = [synthetic.camera_images(scenes[e], a, kind, seed=e * 8 + a) for e, a in b.agents]
    dep = torch.as_tensor(np.stack([f[0] for f in frames])).cuda()
    seg = torch.as_tensor(np.stack([f[1] for f in frames])).cuda()
    dt_e2e = timed(lambda: b.ingest(dep, seg, camera=kind), args.steps, 3)
    prep = b.prepare_ingest(dep, seg, camera=kind)
    for _ in range(3):
        b.launch_ingest(prep)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = max(args.steps, 50)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        b.launch_ingest(prep)
    e1.record(s)
    torch.cuda.synchronize()
    kern_ms = e0.elapsed_time(e1) / steps
    spec = camera.CAMERAS[kind]
    npix = spec.height_px * spec.width_px
    alg = b.N * (8 * npix + 5 * b.H * b.W)
    n, el = 0, 0.0
    for k, (e, a) in enumerate(b.agents):
        sc = scenes[e]
        r = sc['robots'][a]
        ov, oc = sc['overhead'][a].copy(), sc['occupancy'][a].copy()
        t0 = time.perf_counter()
        oracle.ingest(ov, oc, frames[k][0], frames[k][1], spec.params(r['position'][0], r['position'][1], r['heading']),
                      spec, synthetic.SEG_IDS, sc['receptacle_position'] is not None)
        el += time.perf_counter() - t0
        n += 1
        if el > args.cpu_budget:
            break
    print(json.dumps({'row': 'ingest', 'config': args.config, 'camera': kind, 'frames_per_launch': b.N,
                      'points_per_frame': npix, 'gpu_frames_per_s': b.N / (kern_ms * 1e-3),
                      'gpu_ms_per_launch': kern_ms, 'gpu_frames_per_s_end_to_end': b.N / dt_e2e,
                      'gpu_ms_end_to_end': dt_e2e * 1e3,
                      'roofline': {'bound': 'hbm', 'achieved': alg / (kern_ms * 1e-3) / 1e9, 'peak': 8000.0,
                                   'unit': 'GB/s', 'frac': alg / (kern_ms * 1e-3) / 1e9 / 8000.0,
                                   'algorithmic_bytes_per_frame': alg // b.N,
                                   'kernels': 'ingest_points_kernel + ingest_resolve_kernel'},
                      'cpu_oracle_frames_per_s': n / el, 'cpu_cores': 1,
                      'cpu_sample': '%d frames: capture_image points + argsort scatter + obstacle scatter' % n}),
          flush=True)


def bench_mixed(envs=64, steps=50):
    """`envs` envs of each BASELINE configuration (configs[0..4]; pushing_4-large_empty and
    lifting_2_throwing_2-large_empty share one), interleaved env by env, rendered by ONE
    MixedStateBatch launch vs one StateBatch launch per configuration back to back on the same
    stream.  Device time by HIP events over `steps` launches (sequences) after warm-up."""
    cfgs = ['lifting_1-small_empty', 'lifting_4-small_divider', 'pushing_4-large_empty',
            'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty']
    scenes = [synthetic.make_scene(c, 1000 * k + e) for e in range(envs) for k, c in enumerate(cfgs)]
    mb = batch.MixedStateBatch(scenes)
    out = mb.alloc_state()
    groups = {}
    for s in scenes:
        groups.setdefault(batch.config_key(s), []).append(s)
    sbs = [batch.StateBatch(g) for g in groups.values()]
    outs = [b.alloc_state() for b in sbs]
    s = torch.cuda.current_stream()
    res = {}
    for name, f in (('mixed', lambda: mb.render(out)), ('per_config', lambda: [b.render(o) for b, o in zip(sbs, outs)])):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / steps
    got = mb.states(out)
    env_of = {id(sc): i for i, sc in enumerate(scenes)}
    slot = {ea: k for k, ea in enumerate(mb.agents)}
    ok = all(torch.equal(got[slot[(env_of[id(b.scenes[e])], a)]], o[n])
             for b, o in zip(sbs, outs) for n, (e, a) in enumerate(b.agents))
    print(json.dumps({'row': 'mixed', 'configs': cfgs, 'envs_per_config': envs, 'stacks': mb.N,
                      'configurations_in_launch': len(mb.plan['cfgs']),
                      'mixed_ms': res['mixed'], 'per_config_ms': res['per_config'],
                      'mixed_stacks_per_s': mb.N / (res['mixed'] * 1e-3),
                      'per_config_stacks_per_s': mb.N / (res['per_config'] * 1e-3),
                      'per_config_launches': len(sbs), 'mixed_equals_per_config': bool(ok),
                      'note': 'HIP events over %d launches (sequences); inputs resident' % steps}), flush=True)


def bench_gridgraph_large(n=500, density=0.25, seed=505):
    """GridGraph(grid).shortest_path_image / shortest_path on an n x n random grid (obstacle density
    `density`), B = 1, 64 and 256 queries per launch (256: one query per CU), against the oracle's C SPFA (the reference's
    algorithm, 1 core; the reference's Cython SPFA runs at about the same speed, profiles/r2_cpu_calibration.json)."""
    import oracle
    rs = np.random.RandomState(seed)
    grid = (rs.random_sample((n, n)) > density).astype(np.uint8)
    free = np.argwhere(grid != 0)
    pick = lambda k: free[rs.randint(len(free), size=k)].astype(np.int32)  # noqa: E731
    g1 = torch.from_numpy(grid).cuda()
    rows = {}
    for B in (1, 64, 256):
        grids = g1.unsqueeze(0).expand(B, n, n).contiguous()
        srcs = torch.from_numpy(pick(B)).cuda()
        tg = pick(B)
        img = timed(lambda: batch.sssp_grid(grids, srcs), 3, 1)
        pth = timed(lambda: batch.launch_grid_paths(grids, srcs, torch.from_numpy(tg).cuda(), max_points=1024), 2, 1)
        rows[B] = (img, pth)
    s0, t0 = pick(1)[0], pick(1)[0]
    c0 = time.perf_counter()
    oracle.spfa_image(grid, tuple(s0))
    cpu_img = time.perf_counter() - c0
    c0 = time.perf_counter()
    oracle.grid_shortest_path(grid, tuple(s0), tuple(t0))
    cpu_path = time.perf_counter() - c0
    print(json.dumps({'row': 'gridgraph_large', 'grid': '%dx%d' % (n, n), 'obstacle_density': density,
                      'gpu_image_ms': {str(B): v[0] * 1e3 for B, v in rows.items()},
                      'gpu_images_per_s_at_64': 64 / rows[64][0], 'gpu_images_per_s_at_256': 256 / rows[256][0],
                      'gpu_path_ms': {str(B): v[1] * 1e3 for B, v in rows.items()},
                      'gpu_paths_per_s_at_64': 64 / rows[64][1], 'gpu_paths_per_s_at_256': 256 / rows[256][1],
                      'cpu_oracle_image_ms': cpu_img * 1e3, 'cpu_oracle_path_ms': cpu_path * 1e3, 'cpu_cores': 1,
                      'note': 'image: gl_tile_kernel (62 x 62 tiles in LDS, a queue of dirty tiles, four groups '
                              'of four waves; gl_sssp_kernel whole-window sweeps beyond 4,096 tiles); path: that '
                              'fixpoint + gl_path_kernel (one wave replays the SPFA, early exit at the target chain); '
                              'the SPFA is serial, one L2 round trip per pop'}), flush=True)


if __name__ == '__main__':
    if '--mixed' in sys.argv:
        bench_mixed()
        sys.exit(0)
    if '--gridgraph-large' in sys.argv:
        bench_gridgraph_large()
        sys.exit(0)
    if '--env-step' in sys.argv:
        bench_env_step(argparse.Namespace(config='lifting_4-small_divider', envs=64, steps=50, all=False))
        bench_env_step(argparse.Namespace(config='lifting_4-small_divider', envs=64, steps=50, all=True))
        sys.exit(0)
    if '--dropin-only' in sys.argv:
        bench_dropin_step(argparse.Namespace(config='lifting_4-small_divider', envs=64, steps=50))
        bench_remap(argparse.Namespace(config='lifting_4-small_divider', envs=64))
        sys.exit(0)
    if '--ingest-only' in sys.argv:
        sys.argv.remove('--ingest-only')
    else:
        main()
        bench_dropin_step(argparse.Namespace(config='lifting_4-small_divider', envs=64, steps=50))
    bench_ingest(argparse.Namespace(config='lifting_4-small_divider', envs=64, steps=10, cpu_budget=8.0))
