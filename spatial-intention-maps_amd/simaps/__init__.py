"""simaps -- MI355X-native observation-map pipeline of Spatial Intention Maps.

Submodules (imported lazily so that the pure-numpy ones -- constants, synthetic -- stay usable
without torch, e.g. from the python3.9 golden generator):
  constants  reference constants (envs.py)
  synthetic  seeded synthetic scenes
  _lib       ctypes binding of libsimaps.so (the C-ABI in include/simaps.h)
  batch      device-resident batched scene packing + the fused get_state launch
  mapper     drop-ins for the reference's GridGraph / OccupancyMap / Mapper / VectorEnv.get_state
"""
__all__ = ['constants', 'synthetic']
