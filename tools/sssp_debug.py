"""Debug / A-B helper (GPU box): the library named by SIMAPS_LIB against the oracle on the SSSP
users -- sp_distance goldens, sssp_grid on width-92 divider rooms -- with mismatch counts and
kernel times.  Test infrastructure only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import goldens as G  # noqa: E402
import oracle as O  # noqa: E402
from simaps import _lib, batch, synthetic  # noqa: E402
from test_gpu_parity import _room_grids  # noqa: E402


def main():
    res = {'lib': os.environ.get('SIMAPS_LIB', 'default')}
    z = G.load('sp_distance.npz')
    keys = sorted(k[:-len('_dist')] for k in z.files if k.endswith('_dist'))
    by_cfg = {}
    for key in keys:
        cfg, rest = key.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        by_cfg.setdefault(cfg, []).append((e, a, key))
    for cfg, items in by_cfg.items():
        scenes = [synthetic.make_scene(cfg, 40 + e) for e in range(2)]
        b = batch.StateBatch(scenes)
        slots = [b.agents.index((e, a)) for e, a, _ in items]
        src = np.stack([z[k + '_src'] for _, _, k in items])
        tgt = np.stack([z[k + '_queries'] for _, _, k in items])
        got = b.shortest_path_distances(src, tgt, slots=slots).cpu().numpy()
        want = np.stack([z[k + '_dist'] for _, _, k in items])
        bad = got != want
        res['spd_' + cfg] = {'mismatch': int(bad.sum()), 'of': int(bad.size),
                             'max_abs': float(np.abs(got - want).max()),
                             'examples': [[float(a), float(b_)] for a, b_ in zip(got[bad][:4], want[bad][:4])]}
    for h in (44, 92):
        grids, srcs = _room_grids(6, h, 92, 40 + h)
        out = batch.sssp_grid(torch.from_numpy(grids).cuda(), torch.tensor(srcs, dtype=torch.int32),
                              window=(2, 2, h, 92)).cpu().numpy()
        mm = []
        for q in range(len(srcs)):
            ref = O.spfa_image(grids[q], srcs[q])
            d = out[q].view(np.int32) != ref.view(np.int32)
            mm.append(int(d.sum()))
            if d.any() and 'grid_example_%d' % h not in res:
                i, j = np.argwhere(d)[0]
                res['grid_example_%d' % h] = [int(i), int(j), float(out[q][i, j]), float(ref[i, j])]
        res['grid_h%d_mismatch_cells' % h] = mm
    try:
        _lib.check_faults()
        res['faults'] = 0
    except Exception as ex:  # noqa: BLE001
        res['faults'] = str(ex)
    # timing: sssp_grid of 1024 grids h=44, sp_distance 256 x 8
    grids, srcs = _room_grids(1024, 44, 92, 7)
    g = torch.from_numpy(grids).cuda()
    s = torch.tensor(srcs, dtype=torch.int32)
    for _ in range(3):
        batch.sssp_grid(g, s, window=(2, 2, 44, 92))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        batch.sssp_grid(g, s, window=(2, 2, 44, 92))
    e1.record()
    torch.cuda.synchronize()
    res['sssp_grid_h44_1024_us'] = e0.elapsed_time(e1) / 20 * 1e3
    print(json.dumps(res))


if __name__ == '__main__':
    main()
