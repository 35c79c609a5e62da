"""Time OccupancyMap.shortest_path launches (256 agents, lifting_4-small_divider) with the library
named by SIMAPS_LIB: median wall time of batch.shortest_paths (launch + D2H + host unpacking) over
20 calls.  For A/B runs of product builds (tools/prod_build.sh) in one GPU call.  Diagnostic only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
from simaps import batch, synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'lifting_4-small_divider'
scenes = [synthetic.make_scene(cfg, e) for e in range(64)]
b = batch.StateBatch(scenes)
rs = np.random.RandomState(0)
rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
ptgt = np.stack([rs.uniform(0.05, rl / 2, b.N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, b.N)], -1)
out = b.shortest_paths(psrc, ptgt)
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    b.shortest_paths(psrc, ptgt)
    ts.append(time.perf_counter() - t0)
print(json.dumps({'lib': os.path.basename(os.environ.get('SIMAPS_LIB', 'libsimaps.so')), 'config': cfg,
                  'paths': b.N, 'ms_median': float(np.median(ts)) * 1e3,
                  'waypoints_hash': int(sum(len(p) * (k + 1) for k, p in enumerate(out)))}))
