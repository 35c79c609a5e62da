"""Time reward-lookup launches (OccupancyMap.shortest_path_distance, 256 agents x Q targets,
lifting_4-small_divider) with the library named by SIMAPS_LIB: HIP events around 20 launches on the
current stream, inputs resident.  For A/B runs of product builds.  Diagnostic only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import batch, synthetic  # noqa: E402

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 8
scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
b = batch.StateBatch(scenes)
rs = np.random.RandomState(0)
src = torch.as_tensor(np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents]), device='cuda')
tgt = torch.as_tensor(np.stack([rs.uniform(-0.45, 0.45, (b.N, Q)), rs.uniform(-0.2, 0.2, (b.N, Q))], -1), device='cuda')
out = b.shortest_path_distances(src, tgt)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    b.shortest_path_distances(src, tgt)
e1.record()
torch.cuda.synchronize()
print(json.dumps({'lib': os.path.basename(os.environ.get('SIMAPS_LIB', 'libsimaps.so')), 'Q': Q,
                  'us_per_launch': e0.elapsed_time(e1) / 20 * 1e3, 'checksum': float(out.sum())}))
