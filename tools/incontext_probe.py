"""Why get_state_kernel takes longer inside the drop-in step than back to back:
per-launch HIP-event times of the same 256-stack render under different surroundings.

  back_to_back      K renders queued without host gaps (the bench line's loop)
  sync_each         render + synchronize per step, no descriptor update
  gap_<us>          render + synchronize + host spin of <us> (the GPU idles in between)
  update_arrays     update_arrays (H2D of fresh descriptors) + render + synchronize (the drop-in step)
  update_same_buf   as update_arrays but the descriptors are re-uploaded into ONE reused device buffer

GPU box only.  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import batch, synthetic, vector_env  # noqa: E402


def main():
    scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
    arrays = batch.descriptor_arrays(scenes)
    obs = vector_env.VectorEnvObservations(scenes, layout='chw')
    b = obs.batch
    out = b.alloc_state()
    s = torch.cuda.current_stream()
    n = 200

    def timed_launch():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        b.render(out=out)
        e1.record(s)
        return e0, e1

    def spin(us):
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e6 < us:
            pass

    res = {}
    for _ in range(20):
        b.render(out=out)
    torch.cuda.synchronize()
    evs = [timed_launch() for _ in range(n)]
    torch.cuda.synchronize()
    res['back_to_back'] = float(np.median([a.elapsed_time(c) for a, c in evs])) * 1e3
    for name, gap, upd in (('sync_each', 0, None), ('gap_100', 100, None), ('gap_500', 500, None), ('gap_2000', 2000, None),
                           ('update_arrays', 0, 'arrays'), ('update_arrays_gap_500', 500, 'arrays')):
        ts = []
        for _ in range(n):
            if upd:
                obs.update_arrays(**arrays)
            a, c = timed_launch()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(c))
            if gap:
                spin(gap)
        res[name] = float(np.median(ts)) * 1e3
    print(json.dumps({'probe': 'get_state_kernel us per launch (HIP events, median of %d)' % n, **res}), flush=True)


if __name__ == '__main__':
    main()
