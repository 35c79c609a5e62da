"""Does the GPU need sustained work before the timed region reaches its steady per-step time?
(GPU box) A fresh process: 5 warm-up renders, then timed regions of K = 20 and 200 (as bench.py's
timed region: sync, K renders, sync), then ~`--heat` ms of back-to-back renders, then the same
regions again; and the bench's event-bracketed form of each."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import torch  # noqa: E402

from simaps import batch, synthetic  # noqa: E402

heat_ms = float(sys.argv[sys.argv.index('--heat') + 1]) if '--heat' in sys.argv else 300.0
scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
b = batch.StateBatch(scenes)
out = b.alloc_state()
s = torch.cuda.current_stream()


def region(K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        b.render(out, stream=s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6


for _ in range(5):
    b.render(out, stream=s)
res = {'cold': {'K20': region(20), 'K200': region(200), 'K20_again': region(20)}}
t0 = time.perf_counter()
n = 0
while (time.perf_counter() - t0) * 1e3 < heat_ms:
    for _ in range(100):
        b.render(out, stream=s)
    torch.cuda.synchronize()
    n += 100
res['heat'] = {'renders': n, 'ms': (time.perf_counter() - t0) * 1e3}
res['hot'] = {'K20': region(20), 'K200': region(200), 'K20_again': region(20)}
time.sleep(0.5)
res['after_0.5s_idle'] = {'K20': region(20), 'K200': region(200)}
print(json.dumps(res), flush=True)
