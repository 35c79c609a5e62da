"""Debug (GPU box): gl_sssp_kernel images vs the oracle SPFA on a few grids; prints the differing cells."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import numpy as np, torch
import oracle as O, goldens as G
from simaps import batch

def run(name, grid, src):
    H, W = grid.shape
    g = torch.from_numpy(grid).cuda()[None].contiguous()
    img = batch.sssp_grid(g, torch.tensor([src], dtype=torch.int32), window=(0, 0, H, W)).cpu().numpy()[0]
    ref = O.spfa_image(grid, src)
    d = np.argwhere(img.view(np.int32) != ref.view(np.int32))
    print(name, grid.shape, src, 'ndiff', len(d), flush=True)
    for (i, j) in d[:8]:
        print('   ', (int(i), int(j)), 'gpu', float(img[i, j]), 'ref', float(ref[i, j]))
    if len(d):
        gi = img[d[:, 0], d[:, 1]]; ri = ref[d[:, 0], d[:, 1]]
        print('    gpu>ref', int((gi > ri).sum()), 'gpu<ref', int((gi < ri).sum()), 'gpu==-1', int((gi == -1).sum()), 'ref==-1', int((ri == -1).sum()))

print('lib:', os.environ.get('SIMAPS_LIB', 'product'))
g = G.load('sssp.npz')
demo = g['demo_cspace']
run('demo', demo, (75, 156))
run('empty130', np.ones((130, 130), np.uint8), (5, 7))
run('empty70x130', np.ones((70, 130), np.uint8), (5, 7))
run('empty130x70', np.ones((130, 70), np.uint8), (5, 7))
rs = np.random.RandomState(1)
run('rand200', (rs.random_sample((200, 200)) > 0.25).astype(np.uint8), (100, 100))
run('line', np.ones((1, 300), np.uint8), (0, 5))
run('col', np.ones((300, 1), np.uint8), (5, 0))
