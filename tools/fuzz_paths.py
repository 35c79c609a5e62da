"""Diagnostic: GridGraph.shortest_path on tie-heavy random grids vs the oracle (the cases of
tests/test_gpu_dropin.py::test_gridgraph_paths_fuzz_vs_oracle); prints the mismatches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402
from simaps import vector_env  # noqa: E402
from test_gpu_dropin import _tie_grids  # noqa: E402

rs = np.random.RandomState(1234)
bad = n = 0
for gi, grid in enumerate(_tie_grids(rs)):
    free = np.argwhere(grid != 0)
    gg = vector_env.GridGraph(grid)
    srcs = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(4)]
    for src in srcs:
        gg.shortest_path_image(src)
        O.spfa_image(grid, src)
        tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(10)]
        got = gg.shortest_paths([(src, t) for t in tgts])
        for t, p in zip(tgts, got):
            want = O.grid_shortest_path(grid, src, t)
            a, b = np.array(p).reshape(-1, 2), np.array(want).reshape(-1, 2)
            n += 1
            if not np.array_equal(a, b):
                bad += 1
                if bad <= 5:
                    print('grid', gi, grid.shape, 'src', src, 'tgt', t, 'gpu', a.tolist(), 'oracle', b.tolist())
print('mismatches', bad, 'of', n)
