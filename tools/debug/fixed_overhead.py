"""Where the bench's fixed per-region cost goes (GPU box): the timed region (sync, K launches,
sync) for K = 0, 1, 5, 20, 200 -- intercept = fixed cost, slope = per-step time -- with the HIP
runtime's default device scheduling, or with spin-wait synchronisation (--spin: hipSetDeviceFlags
(hipDeviceScheduleSpin) before the device is initialised)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import torch  # noqa: E402

if '--spin' in sys.argv:
    hip = ctypes.CDLL('libamdhip64.so')
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    print('hipSetDeviceFlags(spin) ->', rc, flush=True)

from simaps import batch, synthetic  # noqa: E402

scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
b = batch.StateBatch(scenes)
out = b.alloc_state()
for _ in range(50):
    b.render(out)
torch.cuda.synchronize()
res = {}
for K in (0, 1, 5, 20, 200):
    ts = []
    for rep in range(30 if K <= 20 else 5):
        for _ in range(5):
            b.render(out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            b.render(out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    res[K] = {'median_us': ts[len(ts) // 2] * 1e6, 'min_us': ts[0] * 1e6}
t0 = time.perf_counter()
for _ in range(200):
    torch.cuda.synchronize()
res['idle_sync_us'] = (time.perf_counter() - t0) / 200 * 1e6
print(json.dumps({'spin': '--spin' in sys.argv, 'regions': res}), flush=True)
