"""Per-agent kernel time: each agent rendered alone (one workgroup per launch), HIP-event timed.
Finds the workgroups that set a launch's tail.  Diagnostic only.
    python tools/agent_times.py CONFIG ENVS"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import batch, synthetic  # noqa: E402

cfg, E = sys.argv[1], int(sys.argv[2])
scenes = [synthetic.make_scene(cfg, e) for e in range(E)]
b = batch.StateBatch(scenes)
out = b.alloc_state(1)
res = []
for n in range(b.N):
    for _ in range(2):
        b.render(out, slots=[n])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.render(out, slots=[n])
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / 10 * 1e3)
res = np.array(res)
o = np.argsort(-res)
print(cfg, 'median %.1f us' % np.median(res), 'slowest:', [(int(n), b.agents[n], round(float(res[n]), 1)) for n in o[:10]])
