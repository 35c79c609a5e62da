"""Host-side cost of one StateBatch.render call (Python + ctypes + hipLaunchKernel), and of the same
C-ABI call with its arguments bound once, measured with an idle and with a busy GPU queue; and the
20-step region's fixed cost (first launch + final synchronize) as the bench sees it.

    python tools/debug/host_launch_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import _lib, batch, synthetic  # noqa: E402


def main():
    scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
    b = batch.StateBatch(scenes, device='cuda', layout='chw')
    out = b.alloc_state()
    s = torch.cuda.current_stream()
    for _ in range(50):
        b.render(out, stream=s)
    torch.cuda.synchronize()
    L = _lib.lib
    args = (b.cfg, b.N, _lib.ptr(b.agents_d), _lib.ptr(b.envs_d), _lib.ptr(b.robots_d), _lib.ptr(b.paths_d),
            _lib.ptr(b.occupancy), _lib.ptr(b.overhead), _lib.ptr(out), 0, None, _lib.stream_handle(s))
    res = {}
    for name, fn in (('render', lambda: b.render(out, stream=s)), ('bound', lambda: L.simaps_get_state(*args))):
        idle, busy = [], []
        for _ in range(200):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            idle.append(time.perf_counter() - t)
        torch.cuda.synchronize()
        for _ in range(20):  # keep the queue busy: the next calls return while the GPU works
            fn()
        for _ in range(200):
            t = time.perf_counter()
            fn()
            busy.append(time.perf_counter() - t)
        torch.cuda.synchronize()
        res[name] = {'idle_us_median': 1e6 * float(np.median(idle)), 'busy_us_median': 1e6 * float(np.median(busy))}
        # region fixed cost: K-step regions for K = 1, 20, 200, time per region minus K x per-step slope
        reg = {}
        for K in (1, 2, 20, 200):
            ts = []
            for _ in range(30):
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(K):
                    fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            reg[K] = 1e6 * float(np.median(ts))
        slope = (reg[200] - reg[20]) / 180
        res[name].update({'region_us': reg, 'slope_us_per_step': slope, 'fixed_us': reg[20] - 20 * slope})
    _lib.check_faults()
    print(json.dumps(res))


if __name__ == '__main__':
    main()
