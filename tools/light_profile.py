"""Per-workgroup stamps of the SIMAPS_LIGHT_STAMPS diagnostic build (a few s_memrealtime stamps, no
added barriers): the slowest workgroups' timeline (us from their start).  Diagnostic only.

    SIMAPS_LIB=.../libsimaps_light.so python tools/light_profile.py --config NAME [--envs E]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import _lib, batch, synthetic  # noqa: E402

NAMES = {7: 'sweep_end', 8: 'render_end', 11: 'ovh_robot', 62: 'raster_wait', 60: 'raster_zero', 61: 'raster_lines',
         13: 'raster_end'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-large_rooms')
    ap.add_argument('--envs', type=int, default=16)
    ap.add_argument('--top', type=int, default=8)
    args = ap.parse_args()
    L = _lib.lib
    L.simaps_debug_read_stamps.argtypes = [ctypes.c_void_p]
    scenes = [synthetic.make_scene(args.config, e) for e in range(args.envs)]
    b = batch.StateBatch(scenes)
    out = b.alloc_state()
    for _ in range(3):
        b.render(out)
    torch.cuda.synchronize()
    st = np.zeros((8192, 80), dtype=np.uint64)
    assert L.simaps_debug_read_stamps(st.ctypes.data) == 0
    st = st[:b.N].astype(np.int64)
    rel = (st - st[:, :1]) / 100.0
    order = np.argsort(-rel[:, 8])
    for n in order[:args.top]:
        print(n, b.agents[n], ' '.join('%s %.1f' % (NAMES[k], rel[n, k]) for k in sorted(NAMES, key=lambda k: rel[n, k])))
    print('median', ' '.join('%s %.1f' % (NAMES[k], np.median(rel[:, k])) for k in NAMES))


if __name__ == '__main__':
    main()
