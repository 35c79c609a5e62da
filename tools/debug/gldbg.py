import os, sys
os.environ['SIMAPS_LIB'] = os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'spatial-intention-maps_amd/simaps/libsimaps_gldbg.so')
sys.path.insert(0, 'spatial-intention-maps_amd'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import numpy as np, torch
import goldens as G
from simaps import _lib, batch
demo = G.load('sssp.npz')['demo_cspace']; H, W = demo.shape
z = G.load('grid_paths.npz')
keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))[:4]
pairs = [(tuple(int(x) for x in z[k + '_src']), tuple(int(x) for x in z[k + '_tgt'])) for k in keys]
g = torch.from_numpy(demo).cuda().unsqueeze(0).expand(len(pairs), H, W).contiguous()
for mode in (0, 4, 5):
    _lib.lib.simaps_path_mode(mode)
    got = batch.grid_paths(g, [p[0] for p in pairs], [p[1] for p in pairs], window=(0, 0, H, W), max_points=512)
    torch.cuda.synchronize()
    print('mode', mode, got, flush=True)
