"""Fresh-seed fuzz of GridGraph on windows beyond the LDS limit (the tiled fixpoint, csrc/grid_large.h
gl_tile_kernel, and gl_path_kernel) against the oracle's C SPFA: random sizes (odd tile remainders
included), obstacle densities from open to near-percolation, blocks / corridors / pillar lattices,
sources anywhere (tile corners and seams too), batched 4 sources per launch.  Images must be
bitwise the oracle's; paths equal, or differ only at an approximate_polygon tie.
One JSON line.

    python tools/fuzz_large.py [n_grids] [seed0]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402
from simaps import vector_env  # noqa: E402
from test_gpu_dropin import _dp_tie  # noqa: E402


def make_grid(rs):
    h, w = int(rs.randint(64, 700)), int(rs.randint(121, 700))
    kind = rs.randint(4)
    if kind == 0:  # random cells
        g = (rs.random_sample((h, w)) > rs.uniform(0.0, 0.42)).astype(np.uint8)
    elif kind == 1:  # random rectangles
        g = np.ones((h, w), np.uint8)
        for _ in range(rs.randint(5, 60)):
            i, j = rs.randint(h), rs.randint(w)
            g[i:i + rs.randint(1, 40), j:j + rs.randint(1, 40)] = 0
    elif kind == 2:  # pillar lattice (ties)
        g = np.ones((h, w), np.uint8)
        p = int(rs.randint(3, 9))
        g[p // 2::p, p // 2::p] = 0
    else:  # corridors: walls with gaps every 62 rows / columns (tile seams)
        g = np.ones((h, w), np.uint8)
        for r in range(int(rs.randint(10, 70)), h, int(rs.randint(20, 90))):
            g[r, :] = 0
            g[r, rs.randint(w)] = 1
    return g


def main():
    n_grids = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 80000
    t0 = time.time()
    n_img = bad_img = n_path = tie = bad_path = n_large = 0
    for k in range(n_grids):
        rs = np.random.RandomState(seed0 + k)
        grid = make_grid(rs)
        free = np.argwhere(grid != 0)
        if len(free) < 2:
            continue
        gg = vector_env.GridGraph(grid)
        n_large += bool(gg.large)
        corner = (min(61, grid.shape[0] - 1), min(61, grid.shape[1] - 1))
        srcs = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(3)] + [corner]
        imgs = gg.shortest_path_images(srcs).cpu().numpy()
        for s, img in zip(srcs, imgs):
            n_img += 1
            if not np.array_equal(img.view(np.int32), O.spfa_image(grid, s).view(np.int32)):
                bad_img += 1
                print('IMAGE MISMATCH', seed0 + k, grid.shape, s, file=sys.stderr)
        src = srcs[0]
        tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(3)]
        for t, p in zip(tgts, gg.shortest_paths([(src, t) for t in tgts])):
            n_path += 1
            want = O.grid_shortest_path(grid, src, t)
            if np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
                continue
            if _dp_tie(grid, src, t):
                tie += 1
            else:
                bad_path += 1
                print('PATH MISMATCH', seed0 + k, grid.shape, src, t, file=sys.stderr)
        if k % 16 == 15:
            print('progress %d/%d' % (k + 1, n_grids), file=sys.stderr, flush=True)
    print(json.dumps({'row': 'fuzz_large', 'seeds': [seed0, seed0 + n_grids - 1], 'grids': n_grids,
                      'large_windows': n_large, 'images': n_img, 'image_mismatches': bad_img, 'paths': n_path,
                      'path_ties': tie, 'path_mismatches': bad_path, 'seconds': round(time.time() - t0, 1)}))
    sys.exit(1 if bad_img or bad_path else 0)


if __name__ == '__main__':
    main()
