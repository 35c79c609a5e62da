"""Render ONE agent (map slot) of a config K times -- for per-dispatch counter passes.  Diagnostic.
    python tools/one_agent.py CONFIG ENVS SLOT [K]"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'spatial-intention-maps_amd'))
import torch  # noqa: E402
from simaps import batch, synthetic  # noqa: E402

cfg, E, slot = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
K = int(sys.argv[4]) if len(sys.argv) > 4 else 5
b = batch.StateBatch([synthetic.make_scene(cfg, e) for e in range(E)])
out = b.alloc_state(1)
for _ in range(K):
    b.render(out, slots=[slot])
torch.cuda.synchronize()
print('ok')
