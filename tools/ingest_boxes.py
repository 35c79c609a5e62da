"""Chunk boxes of the ingest point pass (GPU box): per frame, the sum of the chunk boxes' areas
against the area of their bounding box (what ingest_resolve_kernel sweeps), and how many map pixels
the frame really touches (nonzero keys before the resolve).  One JSON line per camera."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from simaps import batch, synthetic  # noqa: E402

for kind in ('forward', 'overhead'):
    scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(16)]
    b = batch.StateBatch(scenes)
    frames = [synthetic.camera_images(scenes[e], a, kind, seed=e * 8 + a) for e, a in b.agents]
    dep = torch.as_tensor(np.stack([f[0] for f in frames])).cuda()
    seg = torch.as_tensor(np.stack([f[1] for f in frames])).cuda()
    b.ingest(dep, seg, camera=kind)
    torch.cuda.synchronize()
    bx = b._boxes.cpu().numpy().reshape(b.N, -1, 4).astype(np.int64)
    areas = (bx[..., 1] - bx[..., 0]) * (bx[..., 3] - bx[..., 2])
    union = (bx[..., 1].max(1) - bx[..., 0].min(1)) * (bx[..., 3].max(1) - bx[..., 2].min(1))
    print(json.dumps({'camera': kind, 'chunks': int(bx.shape[1]), 'map_pixels': b.H * b.W,
                      'sum_chunk_box_area_median': float(np.median(areas.sum(1))),
                      'bounding_box_area_median': float(np.median(union)),
                      'chunk_area_max_median': float(np.median(areas.max(1))),
                      'chunks_over_2048_median': float(np.median((areas > 2048).sum(1))),
                      'chunk_areas_frame0': areas[0].tolist()}), flush=True)
