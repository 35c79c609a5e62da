"""cProfile of the drop-in observation step (VectorEnvObservations.update + get_state) on the GPU
box: where the host time of a step goes.  Diagnostic only."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
import torch  # noqa: E402
from simaps import synthetic, vector_env  # noqa: E402

scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
obs = vector_env.VectorEnvObservations(scenes, layout='chw')


def step():
    obs.update(scenes=scenes)
    obs.get_state()
    torch.cuda.synchronize()


for _ in range(10):
    step()
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    step()
pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
