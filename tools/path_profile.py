"""Per-phase timing of path_kernel (OccupancyMap.shortest_path) from the stamp build
(libsimaps_prof.so): start -> cspace / straight line -> snap -> SPFA init -> SPFA -> parent walk ->
approximate_polygon -> line-of-sight pruning.  Diagnostic only."""
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

cfg = sys.argv[1] if len(sys.argv) > 1 else 'lifting_4-small_divider'
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 64
scenes = [synthetic.make_scene(cfg, e) for e in range(envs)]
b = batch.StateBatch(scenes)
rs = np.random.RandomState(0)
s0 = scenes[0]
rl, rw = s0['room_length'], s0['room_width']
N = b.N
psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
ptgt = np.stack([rs.uniform(0.05, rl / 2, N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, N)], -1)
for _ in range(2):
    b.shortest_paths(psrc, ptgt)
L = _lib.lib
L.simaps_debug_read_stamps.argtypes = [ctypes.c_void_p]
st = np.zeros((8192, 80), dtype=np.uint64)
torch.cuda.synchronize()
assert L.simaps_debug_read_stamps(st.ctypes.data) == 0
st = st[:N].astype(np.int64)
full = st[:, 3] > 0  # ran the SPFA (not a straight line)
us = lambda a, c: [float(np.percentile((st[full, c] - st[full, a]) / 100.0, q)) for q in (50, 90, 100)]  # noqa: E731
print(json.dumps({'config': cfg, 'queries': N, 'spfa_queries': int(full.sum()),
                  'start_to_cspace': us(0, 1), 'snap': us(1, 2), 'spfa_init': us(2, 3) if False else None,
                  'spfa': us(2, 3), 'parent_walk': us(3, 4), 'polygon': us(4, 5), 'prune': us(5, 6),
                  'total': us(0, 6)}, indent=1))
