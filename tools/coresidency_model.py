"""Model: two get_state stacks per CU for launches beyond the CU count.

get_state_kernel runs one 1024-thread workgroup (16 waves) per stack and holds a CU alone: its LDS is
158,864 B and its 123 VGPRs allow 4 waves per SIMD.  Two co-resident stacks need, per stack,
  (a) LDS <= 80 KiB (81,920 B), and
  (b) <= 64 VGPRs (8 waves per SIMD for 2 x 16 waves) -- or 8-wave stacks, which halve each track's
      waves and lengthen its chain, i.e. the same 4 waves per SIMD as today.
This model answers, per BASELINE configuration, from the kernel's own layout constants and from
measurements:
  1. LDS: the smallest layout the data allows -- distance arrays sized to the configuration's room
     (not SIMAPS_MAX_ROOM_CELLS), the raster tile and the robot-code map cut to the pixels the rotated
     96 x 96 sample footprint can touch (the maximum over 3,600 headings of the order-0 source pixels,
     plus the grey-dilation cross for the tile), the descriptor / segment block as today.  Feasible
     iff <= 81,920 B.
  2. Registers: the measured cost of the 64-VGPR budget (the kernel built with amdgpu_waves_per_eu(8, 8)
     and its LDS made dynamic, SIMAPS_VGPR_CAP -- 112 VGPRs and 220 SGPRs spilled, 308 B/lane of
     scratch): per-stack time X = T(64 VGPR) / T(product), both at one workgroup per CU
     (profiles/r6f_v64.jsonl vs profiles/r6f_prod.jsonl).
  3. Contention: the co-resident pair shares each SIMD's issue.  Measured for the SSSP sweep step
     (tools/micro/sweep_mb.hip, round 2, HISTORY.md appendix B): 126 cycles with <= 1 sweep wave per
     SIMD, 148 with 2, 291 with 4 -- the CU saturates at 4 sweep waves per SIMD.  Two stacks double the
     sweep waves per SIMD (lifting: 2 -> 4, rescue: 1 -> 2), so the pair's SSSP rounds take
     rounds_us x step(2k) / step(k), where the stack-alone rounds come from the committed stamp profile.
  Bound on the pair (per 2 stacks, microseconds):  T2 >= max(X * T1, X * (T1 - R) + R * c_sweep)
  with T1 the product's per-stack time at 1,024 stacks (4 workgroups per CU in turn), R the SSSP rounds,
  c_sweep the sweep contention; gain bound = 2 T1 / T2 (perfect overlap of everything else).
  rescue_4-small_empty (configs[4]), the one configuration whose minimal layout fits, is modelled per
  track from its own stamp profile (profiles/r6g_phase_rescue.json): the sweep track (4 waves, 1 -> 2
  per SIMD) and the render track (12 waves, 3 -> 6 per SIMD, contention c_render unmeasured: the
  table's only doubling at >= 2 waves per SIMD is 1.97x) -- the estimate is given as a function of
  c_render, with the break-even values for a 15 % and a 0 % gain.

    python tools/coresidency_model.py > profiles/r6f_coresidency_model.json
"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

LDS_PER_CU = 160 * 1024
BUDGET = LDS_PER_CU // 2
# tools/micro/lds_layout.hip on this tree (get_state_kernel's LDS layout, simaps.hip)
LAYOUT = {'sizeof_Shared': 10488, 'OFF_DIST': 10496, 'DIST_FLOATS': 9024, 'OFF_UNION': 82688,
          'sizeof_SsspScratch': 21248, 'TILE': 138, 'TILE_BYTES': 76176, 'CMAP_BYTES': 18512,
          'UNION_BYTES': 76176, 'LDS_BYTES': 158864, 'CROP': 136, 'LW': 96}
# tools/micro/sweep_mb.hip (round 2): shader cycles per sweep step by sweep waves per SIMD
SWEEP_STEP = {1: 126, 2: 148, 4: 291}
CONFIGS = ['lifting_4-small_divider', 'pushing_4-large_empty', 'lifting_2_throwing_2-large_empty',
           'rescue_4-small_empty']  # BASELINE configs[1]-[4]


def footprint():
    """Max over headings of the crop pixels the 96 x 96 local map samples (order 0), and of those
    plus their 4-neighbours (the intention channel's grey-dilation cross reads the tile there)."""
    import oracle as O
    n, lw = LAYOUT['CROP'], LAYOUT['LW']
    best_s = best_d = 0
    for k in range(3600):
        ang = 90.0 - k * 0.1
        i0, i1, valid = O.rotate_index_map(n, ang)
        S0, S1 = i0.shape
        r0, c0 = S0 // 2 - lw // 2, S1 // 2 - lw // 2
        a, b, v = (x[r0:r0 + lw, c0:c0 + lw] for x in (i0, i1, valid))
        src = set(zip(a[v].tolist(), b[v].tolist()))
        dil = set(src)
        for (i, j) in src:
            dil.update(((i + 1, j), (i - 1, j), (i, j + 1), (i, j - 1)))
        best_s, best_d = max(best_s, len(src)), max(best_d, len(dil))
    return best_s, best_d


def lds_needed(cfg, fp_src, fp_dil):
    from simaps import constants as K, synthetic
    flags = synthetic.config_flags(cfg)
    s = synthetic.make_scene(cfg, 0)
    _, _, h, w = K.room_rect(s['room_width'], s['room_length'])
    nsrc = int(flags['use_shortest_path_to_receptacle_map']) + int(flags['use_shortest_path_map'])
    cells = (h + 2) * ((w + 2) | 1)
    dist = nsrc * cells * 4
    raster = flags['use_intention_map'] or flags['use_history_map']
    # the raster tile (f32 per pixel, exact intention values) aliases the cspace scratch; both are needed
    tile = max(fp_dil * 4 + 138 * 8, LAYOUT['sizeof_SsspScratch']) if raster else LAYOUT['sizeof_SsspScratch']
    # (+ a per-row span table for the compact tile: 138 rows x (offset, first column))
    cmap = fp_src + 138 * 8  # u8 robot-code map over the sampled pixels, same row-span indexing
    today = LAYOUT['LDS_BYTES']
    minimal = LAYOUT['OFF_DIST'] + dist + tile + cmap
    return {'room_rect': [h, w], 'sources': nsrc, 'dist_bytes': dist, 'raster_tile': raster,
            'lds_today': today, 'lds_minimal': minimal, 'fits_two_per_cu': minimal <= BUDGET}


def timings():
    def load(name):
        out = {}
        for line in open(os.path.join(ROOT, 'profiles', name)):
            d = json.loads(line)
            out[(d['config']['workload'], d['config']['stacks_per_step'])] = d['roofline']['kernel_ms'] * 1e3
        return out
    return load('r6f_prod.jsonl'), load('r6f_v64.jsonl')


def main():
    fp_src, fp_dil = footprint()
    prod, v64 = timings()
    phase = json.load(open(os.path.join(ROOT, 'profiles', 'phase_binding.json')))
    rounds_lifting = phase['sweep_track_us']['rounds']
    out = {'lds_budget_per_stack': BUDGET, 'layout': LAYOUT, 'footprint_pixels': fp_src, 'footprint_plus_cross': fp_dil,
           'sweep_step_cycles_by_waves_per_simd': SWEEP_STEP, 'configs': {}}
    for cfg in CONFIGS:
        r = lds_needed(cfg, fp_src, fp_dil)
        if (cfg, 1024) in prod:
            t1 = prod[(cfg, 1024)] / 4  # per stack, 4 workgroups per CU in turn
            X = v64[(cfg, 256)] / prod[(cfg, 256)]
            k = 2 if r['sources'] == 2 else 1  # sweep waves per SIMD today (4 per source over 4 SIMDs)
            c = SWEEP_STEP[2 * k] / SWEEP_STEP[k]
            R = rounds_lifting if cfg == 'lifting_4-small_divider' else None
            t2 = X * t1 if R is None else max(X * t1, X * (t1 - R) + R * c)
            r.update({'t1_us_per_stack_at_1024': t1, 'x_64vgpr_cost': X, 'sweep_contention': c,
                      'sssp_rounds_us': R, 'pair_us_lower_bound': t2, 'gain_upper_bound': 2 * t1 / t2})
        out['configs'][cfg] = r
    # configs[4] per track (its own stamp profile): sweep pair, render pair(c_render), distance phase
    ph = json.load(open(os.path.join(ROOT, 'profiles', 'r6g_phase_rescue.json')))
    r = out['configs']['rescue_4-small_empty']
    X, t1 = r['x_64vgpr_cost'], r['t1_us_per_stack_at_1024']
    c_s = SWEEP_STEP[2] / SWEEP_STEP[1]
    sweep, rounds, render, dist = (ph['sweep_track_us']['end'], ph['sweep_track_us']['rounds'], ph['render_track_us']['end'],
                                   ph['distance_us']['all'])
    sweep_pair = X * (sweep - rounds) * c_s + rounds * c_s
    def pair(c_r):
        return max(sweep_pair, X * render * c_r) + X * dist
    table = {('%.2f' % c): 2 * t1 / pair(c) for c in (1.0, 1.2, 1.4, 1.6, 1.8, 1.97)}
    be = lambda g: (2 * t1 / g - X * dist) / (X * render)  # noqa: E731  c_render at which the gain is g
    r.update({'stamp_profile': {'sweep_track_us': sweep, 'sssp_rounds_us': rounds, 'render_track_us': render,
                                'distance_us': dist, 'source': 'profiles/r6g_phase_rescue.json'},
              'sweep_pair_us': sweep_pair, 'gain_by_render_contention': table,
              'render_contention_for_15pct': be(1.15), 'render_contention_for_break_even': be(1.0)})
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
