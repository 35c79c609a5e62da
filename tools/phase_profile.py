"""Per-phase timing of get_state_kernel from the diagnostic build (libsimaps_prof.so).

Loads the stamp build through SIMAPS_LIB, renders one batch (after a warm-up), and prints per-phase
wall time (median / max over workgroups, us) plus SSSP rounds.  Diagnostic only: the stamps
serialize nothing but add a few instructions; quote shares, not absolute kernel time."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['SIMAPS_LIB'] = os.environ.get('SIMAPS_PROF_LIB', os.path.join(ROOT, 'spatial-intention-maps_amd', 'simaps', 'libsimaps_prof.so'))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from simaps import _lib, batch, synthetic  # noqa: E402

PHASES = ['params+stamps', 'cspace', 'snap+sssp_init', 'split(sweeps || render maps)', 'sssp_finish', 'distance channels']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=64)
    ap.add_argument('--layout', default='chw')
    args = ap.parse_args()
    L = _lib.lib
    L.simaps_debug_read_stamps.argtypes = [ctypes.c_void_p]
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes, layout=args.layout)
    out = b.alloc_state()
    for _ in range(3):
        b.render(out)
    torch.cuda.synchronize()
    st = np.zeros((8192, 48), dtype=np.uint64)
    b.render(out)
    torch.cuda.synchronize()
    assert L.simaps_debug_read_stamps(st.ctypes.data) == 0
    st = st[:b.N].astype(np.int64)
    t = st[:, :7]
    d = np.diff(t, axis=1) / 100.0  # 100 MHz -> us
    sweeps = (st[:, 7] - st[:, 3]) / 100.0
    maps = (st[:, 8] - st[:, 3]) / 100.0
    res = {'config': args.config, 'layout': args.layout, 'N': b.N, 'total_us_median': float(np.median((t[:, 6] - t[:, 0]) / 100.0)),
           'span_us': float((t[:, 6].max() - t[:, 0].min()) / 100.0),
           'split_groups_us': {'sweeps_median': float(np.median(sweeps)), 'render_maps_median': float(np.median(maps)),
                               'sampleidx_raster_gathers': float(np.median((st[:, 14] - st[:, 3]) / 100.0)),
                               'intention_sample': float(np.median((st[:, 13] - st[:, 14]) / 100.0)),
                               'overhead_robot_consume': float(np.median((st[:, 11] - st[:, 13]) / 100.0)),
                               'rest': float(np.median((st[:, 8] - st[:, 11]) / 100.0))},
           'pre_split_us': {'robot_params': float(np.median((st[:, 9] - st[:, 0]) / 100.0)),
                            'stamp_tiles': float(np.median((st[:, 1] - st[:, 9]) / 100.0)),
                            'cspace_stage': float(np.median((st[:, 15] - st[:, 1]) / 100.0)),
                            'cspace_bits': float(np.median((st[:, 2] - st[:, 15]) / 100.0))},
           'distance_us': {'values': float(np.median((st[:, 16] - st[:, 5]) / 100.0)),
                           'block_min': float(np.median((st[:, 17] - st[:, 16]) / 100.0)),
                           'stores': float(np.median((st[:, 6] - st[:, 17]) / 100.0))},
           'sweep_rounds_us': {'round_%d' % r: float(np.median((st[:, 19 + r] - st[:, 18 + r]) / 100.0)) for r in range(3)},
           'first_sweep_us': {'down(w0)': float(np.median((st[:, 22] - st[:, 18]) / 100.0)),
                              'right(w2)': float(np.median((st[:, 23] - st[:, 18]) / 100.0))},
           'wave_sweep_r0_us': {'start': [float(np.median((st[:, 32 + w] - st[:, 18]) / 100.0)) for w in range(8)],
                                'end': [float(np.median((st[:, 24 + w] - st[:, 18]) / 100.0)) for w in range(8)]},
           'render_front_us': {'sampleidx_fast': float(np.median((st[:, 40] - st[:, 3]) / 100.0)),
                               'sampleidx_fp64': float(np.median((st[:, 41] - st[:, 40]) / 100.0)),
                               'raster1': float(np.median((st[:, 42] - st[:, 41]) / 100.0)),
                               'gather_issue': float(np.median((st[:, 14] - st[:, 42]) / 100.0))},
           'rounds': {'median': float(np.median(st[:, 10])), 'max': int(st[:, 10].max()), 'min': int(st[:, 10].min())},
           'phases_us': {p: {'median': float(np.median(d[:, i])), 'max': float(d[:, i].max())}
                         for i, p in enumerate(PHASES)}}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
