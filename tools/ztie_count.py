"""How often the ingest z-tie caveat can matter: over synthetic frames, the touched map
pixels whose highest point is tied in z with another point of that pixel, and among those the ones
where the tied points carry different seg values (only there does the reference's unspecified
np.argsort order change the overhead value).  CPU only, numpy float32 like the oracle.
    python tools/ztie_count.py"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
from simaps import camera as cm, synthetic  # noqa: E402

PPM = 96
tot = ties = diff = 0
for cfg, kind in [('lifting_4-small_divider', 'forward'), ('pushing_4-large_empty', 'forward'),
                  ('lifting_4-small_divider', 'overhead')]:
    for e in range(8):
        s = synthetic.make_scene(cfg, e)
        for a in range(4):
            dep, segraw = synthetic.camera_images(s, a, kind, seed=e * 8 + a)
            spec, r = cm.CAMERAS[kind], s['robots'][a]
            P = spec.params(r['position'][0], r['position'][1], r['heading'])
            Hc, Wc = dep.shape
            depth = spec.far * spec.near / (spec.far - (spec.far - spec.near) * dep)
            cp = np.array(P[0:3], np.float32)
            pr = np.array(P[3:6], np.float32) - cp
            pr = pr / np.linalg.norm(pr)
            cu = np.array(P[6:9], np.float32)
            up = cu - np.dot(cu, pr) * pr
            up = up / np.linalg.norm(up)
            rt = np.cross(pr, up)
            rt = rt / np.linalg.norm(rt)
            ly = math.tan(math.radians(30))
            px = (2 * ly * spec.aspect) * (np.arange(Wc, dtype=np.float32) / Wc - 0.5)
            py = (2 * ly) * (0.5 - (np.arange(Hc, dtype=np.float32) + 1) / Hc)
            pxv, pyv = np.meshgrid(px, py)
            pts = (cp + depth[:, :, None] * (pr + pxv[:, :, None] * rt + pyv[:, :, None] * up)).reshape(-1, 3)
            ids, sr = synthetic.SEG_IDS, segraw.reshape(-1)
            seg = (0.125 * (sr == 0) + 0.25 * ((sr >= ids['min_obstacle']) & (sr <= ids['max_obstacle']))
                   + 0.375 * (sr == ids['receptacle']) + 0.5 * ((sr >= ids['min_cube']) & (sr <= ids['max_cube'])))
            H, W = s['H'], s['W']
            i = np.clip(np.floor(H / 2 - pts[:, 1] * PPM), 0, H - 1).astype(np.int64)
            j = np.clip(np.floor(W / 2 + pts[:, 0] * PPM), 0, W - 1).astype(np.int64)
            pix, z = i * W + j, pts[:, 2]
            o = np.lexsort((z, pix))
            ps, zs, ss = pix[o], z[o], seg[o]
            for k in np.nonzero(np.r_[ps[1:] != ps[:-1], True])[0]:
                tot += 1
                m, n, segs = k - 1, 1, {ss[k]}
                while m >= 0 and ps[m] == ps[k] and zs[m] == zs[k]:
                    n, m = n + 1, m - 1
                    segs.add(ss[m + 1])
                ties += n > 1
                diff += len(segs) > 1
print({'touched_pixels': tot, 'max_z_ties': int(ties), 'ties_with_different_seg': int(diff), 'frames': 96})
