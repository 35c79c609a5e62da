"""The tiled large-window fixpoint's algorithm (csrc/grid_large.h gl_tile_kernel), on the host:
tools/tile_sssp_model.py restates it (dirty-tile queue, halo relaxation of the edge cells, sweep
rounds to each tile's local fixpoint, marks on the neighbours whose halo fell).  With small tiles
(many seams) it reaches the oracle SPFA's image (shortest_paths.pyx:69-114) bit for bit."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import oracle as O  # noqa: E402
import tile_sssp_model as T  # noqa: E402


@pytest.mark.parametrize('tt', [5, 16, 62])
def test_tiled_fixpoint_equals_the_oracle(tt):
    rs = np.random.RandomState(tt)
    grids = [(rs.random_sample((70, 90)) > 0.3).astype(np.uint8), (rs.random_sample((33, 120)) > 0.45).astype(np.uint8)]
    m = np.ones((65, 80), np.uint8)                                    # serpentine
    m[::8, 1:] = 0
    m[4::16, :-1] = 1
    grids.append(m)
    sp = np.zeros((60, 60), np.uint8)                                  # spiral corridor, 1-cell walls
    top, left, bot, right = 0, 0, 59, 59
    sp[0, :] = 1
    while bot - top >= 2 and right - left >= 2:
        sp[top:bot + 1, right] = 1
        sp[bot, left:right + 1] = 1
        sp[top + 2:bot + 1, left] = 1
        top += 2
        sp[top, left:right - 1] = 1
        left, right, bot = left + 2, right - 2, bot - 2
    grids.append(sp)
    for grid in grids:
        free = np.argwhere(grid != 0)
        for src in (tuple(free[0]), tuple(free[rs.randint(len(free))]), tuple(free[-1])):
            img, st = T.tiled_image(grid, src, tt)
            assert np.array_equal(img.view(np.int32), O.spfa_image(grid, src).view(np.int32)), (tt, grid.shape, src)
            assert st['tiles'] >= 1
    blocked = tuple(np.argwhere(grids[0] == 0)[0])
    img, st = T.tiled_image(grids[0], blocked, tt)
    assert img is None and st['tiles'] == 0  # (the kernel then writes 0 at the source, -1 elsewhere)
