"""Movement-path throughput (OccupancyMap.shortest_path, simaps_shortest_path) by launch size, GPU box.

For each (config, envs): robot position -> a target across x = 0 (detours around the divider), all
inputs resident; the device half alone, timed with HIP events on the launch stream over K launches.
With --stamps (the stamp build libsimaps_prof.so) also the per-query SPFA time and pops, i.e. ns per
pop.  One JSON line per launch size.

    python tools/path_bench.py [--stamps]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if '--stamps' in sys.argv:
    os.environ['SIMAPS_LIB'] = os.environ.get('SIMAPS_PROF_LIB', os.path.join(ROOT, 'spatial-intention-maps_amd', 'simaps',
                                                                                'libsimaps_prof.so'))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import _lib, batch, synthetic  # noqa: E402


def case(cfg, envs, steps, mode=0, targets='across'):
    """targets: 'across' -- a random point on the other side of x = 0 (around the divider, if any);
    'local' -- a random point of the robot's own 96 x 96 local map (the action space of
    Robot.store_new_action, envs.py:857-876), clipped to the room."""
    scenes = [synthetic.make_scene(cfg, e % 64) for e in range(envs)]
    b = batch.StateBatch(scenes)
    rs = np.random.RandomState(0)
    rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
    N = b.N
    psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    if targets == 'across':
        ptgt = np.stack([rs.uniform(0.05, rl / 2, N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, N)], -1)
    else:
        ptgt = psrc + rs.uniform(-0.5, 0.5, (N, 2))
        ptgt[:, 0] = np.clip(ptgt[:, 0], -rl / 2 + 0.02, rl / 2 - 0.02)
        ptgt[:, 1] = np.clip(ptgt[:, 1], -rw / 2 + 0.02, rw / 2 - 0.02)
    prev = _lib.lib.simaps_path_mode(mode)
    src = torch.as_tensor(psrc).cuda()
    tgt = torch.as_tensor(ptgt).cuda()
    for _ in range(2):
        b.launch_shortest_paths(src, tgt)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        xy, cnt = b.launch_shortest_paths(src, tgt)
    e1.record(s)
    torch.cuda.synchronize()
    _lib.check_faults()
    _lib.lib.simaps_path_mode(prev)
    ms = e0.elapsed_time(e1) / steps
    out = {'config': cfg, 'targets': targets, 'path_mode': {0: 'auto', 1: 'compact', 2: 'early_exit', 3: 'overlap'}[mode],
           'paths_per_launch': N, 'ms_per_launch': ms, 'paths_per_s': N / (ms * 1e-3),
           'detours': int((cnt.cpu().numpy() > 2).sum())}
    if '--stamps' in sys.argv:
        L = _lib.lib
        L.simaps_debug_read_stamps.argtypes = [ctypes.c_void_p]
        st = np.zeros((8192, 80), dtype=np.uint64)
        assert L.simaps_debug_read_stamps(st.ctypes.data) == 0
        st = st[:min(N, 8192)].astype(np.int64)
        full = st[:, 3] > st[:, 0]  # ran the SPFA in this launch (stale stamps of earlier cases are older)
        spfa_us = (st[full, 3] - st[full, 2]) / 100.0  # s_memrealtime: 100 MHz
        pops = st[full, 7]
        qus = (st[full, 6] - st[full, 0]) / 100.0
        # every query of the launch whose end stamp is from this launch (straight lines end before it)
        allq = np.where(st[:N, 6] > st[:N, 0], st[:N, 6] - st[:N, 0], 0) / 100.0
        t0 = st[:N, 0]
        out.update({'spfa_queries': int(full.sum()), 'spfa_us_median': float(np.median(spfa_us)),
                    'pops_median': float(np.median(pops)), 'pops_max': int(pops.max()) if len(pops) else 0,
                    'query_us_max': float(allq.max()),
                    # latency accounting: the launch lasts as long as its slowest query
                    # plus the dispatch of the workgroups and the kernel's launch / completion overhead
                    'launch_over_slowest_query': ms * 1e3 / float(allq.max()),
                    'slowest_over_median_query': float(allq.max() / np.median(qus)) if len(qus) else None,
                    'entry_skew_us': float((t0.max() - t0.min()) / 100.0),
                    'slowest_query_pops': int(st[:N, 7][np.argmax(allq)]),
                    'sweep_rounds_median': float(np.median(st[full, 8])) if mode in (2, 3) else None,
                    'sweeps_us_median': float(np.median((st[full, 10] - st[full, 2]) / 100.0)) if mode in (2, 3) else None,
                    'ns_per_pop_median': float(np.median(spfa_us * 1e3 / np.maximum(pops, 1))),
                    'query_us_median': float(np.median((st[full, 6] - st[full, 0]) / 100.0))})
    print(json.dumps(out), flush=True)
    return out


if __name__ == '__main__':
    if '--latency' in sys.argv:  # the bench_extra latency row: 64 / 256 paths, local and across, auto mode
        for targets in ('local', 'across'):
            for envs in (16, 64):
                case('lifting_4-small_divider', envs, 5, 0, targets)
        sys.exit(0)
    # (pushing_4-large_empty has no obstacles: nearly all its paths are straight lines, and a launch
    # lasts as long as its slowest query -- a snapped end's full-room SPFA; lifting_4-large_doors:
    # large rooms with detours)
    steps = 5 if '--stamps' in sys.argv else 10
    for targets in ('across', 'local'):
        for cfg, envs in (('lifting_4-small_divider', 16), ('lifting_4-small_divider', 64), ('lifting_4-small_divider', 128),
                          ('lifting_4-small_divider', 256), ('lifting_4-small_divider', 512),
                          ('lifting_4-large_doors', 16), ('lifting_4-large_doors', 64), ('lifting_4-large_doors', 256),
                          ('lifting_4-large_doors', 512)):
            for mode in (1, 2, 3):
                case(cfg, envs, steps, mode, targets)
