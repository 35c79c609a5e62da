"""Where the bench's fixed per-region cost goes (GPU box): the timed region (sync, K launches,
sync) for K = 0, 1, 5, 20, 200 -- intercept = fixed cost, slope = per-step time -- bare and with
the bench's two timing events around the K launches (events_K), with the HIP
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
s = torch.cuda.current_stream()
for events in (False, True):
    for K in (0, 1, 5, 20, 200):
        if events and K == 0:
            continue
        ts = []
        for rep in range(30 if K <= 20 else 5):
            for _ in range(5):
                b.render(out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            for k in range(K):
                if events and k == 0:
                    e0.record(s)
                b.render(out, stream=s)
                if events and k == K - 1:
                    e1.record(s)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        res[('events_' if events else '') + str(K)] = {'median_us': ts[len(ts) // 2] * 1e6, 'min_us': ts[0] * 1e6}
t0 = time.perf_counter()
for _ in range(200):
    torch.cuda.synchronize()
res['idle_sync_us'] = (time.perf_counter() - t0) / 200 * 1e6
print(json.dumps({'spin': '--spin' in sys.argv, 'regions': res}), flush=True)
