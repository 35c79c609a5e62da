"""Pops and cycles of one large-grid path (the gridgraph_large bench's B = 1 query) under a stats
build of gl_path_kernel (-DSIMAPS_GL_STATS: the kernel printfs its pops and the cycles of its pop
loop).  Run with SIMAPS_LIB=<stats build>.  (Round 5 also measured a pipelined pop this way, commit
5a28ec7: profiles/r5m_gl_pop_stats.txt.)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import torch  # noqa: E402

from simaps import batch  # noqa: E402

n, density = 500, 0.25
rs = np.random.RandomState(505)
grid = (rs.random_sample((n, n)) > density).astype(np.uint8)
free = np.argwhere(grid != 0)
pick = lambda k: free[rs.randint(len(free), size=k)].astype(np.int32)  # noqa: E731
g1 = torch.from_numpy(grid).cuda().unsqueeze(0).contiguous()
srcs = torch.from_numpy(pick(1)).cuda()
tg = pick(1)
batch.launch_grid_paths(g1, srcs, torch.from_numpy(tg).cuda(), max_points=1024)
torch.cuda.synchronize()
