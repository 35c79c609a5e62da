"""Parity fuzz of observation ingest on fresh seeds (GPU box): every agent of E envs per
(configuration, camera) takes one synthetic frame through simaps_ingest (one launch), then its
overhead / occupancy maps are compared bitwise with the CPU oracle's Mapper.update + obstacle
scatter (process pool; z ties resolved 'later camera pixel wins' on both sides, as in the tests).

    python tools/fuzz_ingest.py [envs_per_config] [procs]
"""
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

CASES = [('lifting_4-small_divider', 'forward'), ('pushing_4-large_empty', 'forward'), ('rescue_4-small_empty', 'forward'),
         ('lifting_4-large_doors', 'forward'), ('lifting_4-small_divider', 'overhead'), ('lifting_4-large_rooms', 'overhead')]
SEED0 = int(os.environ.get('SIMAPS_FUZZ_SEED0', '7000'))  # (inherited by the spawned oracle workers)


def _oracle(job):
    import oracle as O
    from simaps import camera, synthetic
    cfg, kind, e, a = job
    s = synthetic.make_scene(cfg, SEED0 + e)
    dep, seg = synthetic.camera_images(s, a, kind, seed=SEED0 + 8 * e + a)
    spec, r = camera.CAMERAS[kind], s['robots'][a]
    ov, oc = s['overhead'][a].copy(), s['occupancy'][a].copy()
    O.ingest(ov, oc, dep, seg, spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
             s['receptacle_position'] is not None)
    return ov, oc


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    from simaps import batch, synthetic
    tot = {'frames': 0, 'mismatches': 0}
    with get_context('spawn').Pool(procs) as pool:
        for cfg, kind in CASES:
            t0 = time.time()
            scenes = [synthetic.make_scene(cfg, SEED0 + e) for e in range(envs)]
            b = batch.StateBatch(scenes)
            frames = [synthetic.camera_images(scenes[e], a, kind, seed=SEED0 + 8 * e + a) for e, a in b.agents]
            b.ingest(np.stack([f[0] for f in frames]), np.stack([f[1] for f in frames]), camera=kind)
            ov, oc = b.overhead.cpu().numpy(), b.occupancy.cpu().numpy()
            ep = set(int(x) for x in np.unique(b._keys.cpu().numpy().view(np.uint64) >> np.uint64(56)))
            keys_zero = max(ep) <= b._epoch  # keys untouched or of this or an earlier launch's epoch
            refs = pool.map(_oracle, [(cfg, kind, e, a) for e, a in b.agents], chunksize=2)
            bad = sum(not (np.array_equal(ov[n].view(np.int32), ro.view(np.int32)) and np.array_equal(oc[n], rc))
                      for n, (ro, rc) in enumerate(refs))
            changed = sum(not np.array_equal(ov[n], scenes[e]['overhead'][a]) for n, (e, a) in enumerate(b.agents))
            tot['frames'] += len(refs)
            tot['mismatches'] += bad
            print(json.dumps({'config': cfg, 'camera': kind, 'frames': len(refs), 'mismatches': bad,
                              'maps_changed': changed, 'keys_epochs_ok': keys_zero, 's': round(time.time() - t0, 1)}),
                  flush=True)
    tot['seeds'] = [SEED0, SEED0 + envs - 1]
    print(json.dumps(tot), flush=True)


if __name__ == '__main__':
    main()
