"""Host cost of one get_state launch (GPU box): CPU microseconds per StateBatch.render() call and per
bare simaps_get_state call with pre-built arguments, timed over back-to-back launches without a
synchronize in between (the GPU queue absorbs them).  If a launch costs the host more than the
kernel lasts (~31 us), the bench's timed region is host-bound.  Test infrastructure only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import torch  # noqa: E402

from simaps import _lib, batch, synthetic  # noqa: E402


def per_call(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def main():
    scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
    b = batch.StateBatch(scenes)
    out = b.alloc_state()
    s = torch.cuda.current_stream()
    for _ in range(20):
        b.render(out, stream=s)
    res = {}
    for name, fn in (('render_stream', lambda: b.render(out, stream=s)), ('render_default', lambda: b.render(out))):
        host, wall = per_call(fn, 400)
        res[name] = {'host_us_per_call': host, 'wall_us_per_call': wall}
    args = (b.cfg, b.N, _lib.ptr(b.agents_d), _lib.ptr(b.envs_d), _lib.ptr(b.robots_d), _lib.ptr(b.paths_d),
            _lib.ptr(b.occupancy), _lib.ptr(b.overhead), _lib.ptr(out), 0, None, _lib.stream_handle(s))
    L = _lib.lib
    host, wall = per_call(lambda: L.simaps_get_state(*args), 400)
    res['bare_c_call'] = {'host_us_per_call': host, 'wall_us_per_call': wall}
    t0 = time.perf_counter()
    for _ in range(2000):
        torch.cuda.current_stream()
    res['torch_current_stream_us'] = (time.perf_counter() - t0) / 2000 * 1e6
    print(json.dumps(res))


if __name__ == '__main__':
    main()
