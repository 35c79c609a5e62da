"""PCIe-inclusive get_state rate (the drop-in returning host NumPy arrays, like the reference) beside
the device-resident rate, GPU box.  256 stacks (lifting_4-small_divider, 64 envs x 4 agents), median
wall time per call over 50 calls after 5 warm-up calls:

  device_ring   get_state() into the device output ring (reuse_outputs=2), + synchronize
  numpy_fresh   get_state(numpy=True): a fresh pageable host copy per call (reference semantics)
  numpy_ring    get_state(numpy=True) with reuse_outputs=2: async copy into a pinned host ring
  d2h_pinned    the device->host copy of one rendered batch alone, into pinned memory

    python tools/pcie_rate.py [layout]        (layout: chw (default) or hwc)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import synthetic, vector_env  # noqa: E402


def timed(fn, steps=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main(layout):
    cfg = 'lifting_4-small_divider'
    scenes = [synthetic.make_scene(cfg, e) for e in range(64)]
    plain = vector_env.VectorEnvObservations(scenes, layout=layout)
    ring = vector_env.VectorEnvObservations(scenes, layout=layout, reuse_outputs=2)
    n = plain.batch.N
    buf = plain.batch.render()
    host = torch.empty(buf.shape, dtype=buf.dtype, pin_memory=True)
    cases = {
        'device_ring': lambda: ring.get_state(),
        'numpy_fresh': lambda: plain.get_state(numpy=True),
        'numpy_ring': lambda: ring.get_state(numpy=True),
        'd2h_pinned': lambda: host.copy_(buf, non_blocking=True),
    }
    nbytes = buf.numel() * buf.element_size()
    for name, fn in cases.items():
        s = timed(fn)
        line = {'case': name, 'config': cfg, 'layout': layout, 'stacks': n, 'ms_per_call': s * 1e3,
                'stacks_per_s': n / s, 'state_bytes': nbytes}
        if name != 'device_ring':
            line['d2h_GB_per_s_equiv'] = nbytes / s / 1e9
        print(json.dumps(line), flush=True)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'chw')
