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



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=64)
    ap.add_argument('--layout', default='chw')
    ap.add_argument('--dump', default=None, help='save the raw per-workgroup stamp table (.npy)')
    args = ap.parse_args()
    L = _lib.lib
    L.simaps_debug_read_stamps.argtypes = [ctypes.c_void_p]
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes, layout=args.layout)
    out = b.alloc_state()
    for _ in range(3):
        b.render(out)
    torch.cuda.synchronize()
    st = np.zeros((8192, 80), dtype=np.uint64)
    b.render(out)
    torch.cuda.synchronize()
    assert L.simaps_debug_read_stamps(st.ctypes.data) == 0
    st = st[:b.N].astype(np.int64)
    if args.dump:
        np.save(args.dump, st)
    def us(k1, k0):
        """median over workgroups of stamp k1 - stamp k0 (us); workgroups that recorded neither are
        left out, and a pair no workgroup recorded (a phase this build / config skips) is None."""
        m = (st[:, k1] > 0) & (st[:, k0] > 0)
        return float(np.median((st[m, k1] - st[m, k0]) / 100.0)) if m.any() else None
    res = {'config': args.config, 'layout': args.layout, 'N': b.N,
           'total_us_median': us(6, 0), 'span_us': float((st[:, 6].max() - st[:, 0].min()) / 100.0),
           'sweep_track_us': {'agent_load': us(43, 0), 'first_ballot': us(46, 43), 'all_ballots': us(47, 46), 'v2_ballots_sync': us(15, 47), 'cspace_loads_ballots': us(15, 0), 'cspace_dilate': us(2, 15), 'cspace': us(2, 0), 'snap': us(48, 2), 'init': us(3, 48), 'rounds': us(49, 3), 'finish': us(50, 49), 'scale': us(7, 50), 'rounds_finish_scale': us(7, 3), 'end': us(7, 0)},
           'render_track_us': {'params': us(9, 0), 'blocksets': us(51, 9), 'stamp_tiles': us(1, 51), 'sampleidx_fast': us(40, 1), 'sampleidx_fp64': us(41, 40),
                               'gather_issue': us(42, 41), 'code_lookup': us(14, 42), 'overhead_robot': us(11, 14),
                               'raster_sync_wait': us(62, 11), 'raster_zero_sync': us(60, 62), 'raster_lines': us(61, 60), 'raster_endsync': us(13, 61), 'raster1': us(13, 11), 'sample_rest': us(8, 13), 'end': us(8, 0)},
           'params_us': {'rot_crop': us(72, 0), 'robot0': us(73, 0), 'seg_table0': us(74, 0), 'cmap_zero_w0': us(75, 0)},
           'join_us': us(4, 0),
           'distance_us': {'values': us(16, 5), 'block_min': us(17, 16), 'stores': us(6, 17), 'all': us(6, 5)},
           'sweep_rounds_us': {'round_%d' % r: us(19 + r, 18 + r) for r in range(3)},
           'check_r0_us': {'w0_sweep_end': us(24, 18), 'w3_sweep_end': us(27, 18), 'check_start': us(56, 18),
                           'w0_check_end': us(57, 18), 'w3_check_end': us(63, 18), 'after_barrier': us(78, 18)},
           'wave_sweep_r0_us': {'start': [us(32 + w, 18) for w in range(8)], 'end': [us(24 + w, 18) for w in range(8)]},
           'clock_mhz_sweep_w0': float(np.median((st[:, 45] - st[:, 44]) / ((st[:, 24] - st[:, 18]) / 100.0)))
           if (st[:, 45] > 0).any() else None,
           'dilate_clk_from52': {str(k): float(np.median(st[:, k].astype(np.int64) - st[:, 52].astype(np.int64)))
                                 for k in (53, 54, 55, 56, 57, 58, 59) if (st[:, k] > 0).any()},
           'spread_us': {name: [float(np.percentile((st[:, k1].astype(np.int64) - st[:, 0].astype(np.int64)) / 100.0, q)) for q in (10, 50, 90, 100)]
                         for name, k1 in (('sweep_end', 7), ('render_end', 8), ('join', 4), ('total', 6))},
           'start_skew_us': float((np.percentile(st[:, 0], 100) - np.percentile(st[:, 0], 0)) / 100.0),
           'entry_skew_us': [float(np.percentile((st[:, 77] - st[:, 77].min()) / 100.0, q)) for q in (10, 50, 90, 100)],
           'entry_to_stamp0_us': [float(np.percentile((st[:, 0] - st[:, 77]) / 100.0, q)) for q in (10, 50, 90, 100)],
           'end_after_first_entry_us': [float(np.percentile((st[:, 6] - st[:, 77].min()) / 100.0, q)) for q in (10, 50, 90, 100)],
           'sweep_steps_per_wave': [float(np.median(st[:, 64 + w].astype(np.int64))) for w in range(8)],
           'rounds': {'median': float(np.median(st[:, 10])), 'max': int(st[:, 10].max()), 'min': int(st[:, 10].min())}}
    # SSSP edge relaxations per stack -- every cell of a swept line evaluates its 3
    # incoming edges; wave w of source s sweeps direction (w + 2 s) & 3 (0 / 1: lines of w cells)
    h, w = b.cfg.room_h, b.cfg.room_w
    per_wave = np.median(st[:, 64:72].astype(np.float64), axis=0)
    res['sssp_relaxations_per_stack'] = float(sum(n * (w if ((k + 2 * (k >> 2)) & 3) < 2 else h) * 3
                                                  for k, n in enumerate(per_wave)))
    # drop the phases this build / config never stamped
    res = {k: ({q: v for q, v in d.items() if v is not None} if isinstance(d, dict) else d) for k, d in res.items()}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
