"""Split-sweep SSSP A/B, GPU box: kernel time of the single-source SSSP users --
simaps_sssp_grid (GridGraph.shortest_path_image) and simaps_sp_distance (reward lookups) -- for the
library SIMAPS_LIB points at (a build with -DSIMAPS_SSSP_SPLIT_L / _S, or the product).

    SIMAPS_LIB=.../libsimaps_prod_l2s1.so python tools/sssp_split_ab.py

Rooms 92 cells wide (pitch 95, where the split applies): h = 44 (small rooms) and h = 92 (large),
a divider with one gap.  HIP events on the launch stream around K launches; one JSON line per case.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import batch, synthetic  # noqa: E402


def room_grids(n, h, w, seed):
    rs = np.random.RandomState(seed)
    grids, srcs = [], []
    for _ in range(n):
        g = np.zeros((h + 4, w + 4), np.uint8)
        g[2:2 + h, 2:2 + w] = 1
        c = 2 + w // 2 + rs.randint(-8, 9)
        g[2:2 + h, c] = 0
        gap = 2 + rs.randint(0, h - 6)
        g[gap:gap + 5, c] = 1
        for _ in range(12):
            i, j = 2 + rs.randint(0, h - 4), 2 + rs.randint(0, w - 4)
            g[i:i + rs.randint(1, 5), j:j + rs.randint(1, 5)] = 0
        fr = np.argwhere(g > 0)
        grids.append(g)
        srcs.append(tuple(int(x) for x in fr[rs.randint(len(fr))]))
    return np.stack(grids), srcs


def timed(fn, steps=20, warmup=3):
    for _ in range(warmup):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    lib = os.path.basename(os.environ.get('SIMAPS_LIB', 'libsimaps.so'))
    for h in (44, 92):
        for B in (256, 1024):
            grids, srcs = room_grids(B, h, 92, h)
            g = torch.from_numpy(grids).cuda()
            s = torch.tensor(srcs, dtype=torch.int32)
            out = batch.sssp_grid(g, s, window=(2, 2, h, 92))
            chk = float(out[out > 0].double().sum())
            ms = timed(lambda: batch.sssp_grid(g, s, window=(2, 2, h, 92)))
            print(json.dumps({'lib': lib, 'row': 'sssp_grid', 'h': h, 'w': 92, 'grids': B, 'ms': ms,
                              'us_per_256': ms * 1e3 * 256 / B, 'checksum': chk}), flush=True)
    for cfg in ('lifting_4-small_divider', 'lifting_4-large_doors'):
        scenes = [synthetic.make_scene(cfg, e) for e in range(64)]
        b = batch.StateBatch(scenes)
        rs = np.random.RandomState(0)
        rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
        src = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
        tgt = np.stack([rs.uniform(-rl / 2, rl / 2, (b.N, 8)), rs.uniform(-rw / 2, rw / 2, (b.N, 8))], -1)
        src_d, tgt_d = torch.as_tensor(src).cuda(), torch.as_tensor(tgt).cuda()
        d = b.shortest_path_distances(src_d, tgt_d)
        ms = timed(lambda: b.shortest_path_distances(src_d, tgt_d))
        print(json.dumps({'lib': lib, 'row': 'sp_distance', 'config': cfg, 'agents': b.N, 'ms': ms,
                          'checksum': float(d.sum())}), flush=True)


if __name__ == '__main__':
    main()
