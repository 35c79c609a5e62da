"""simaps -- MI355X-native observation-map pipeline of Spatial Intention Maps.

Submodules (imported lazily so that the pure-numpy ones -- constants, synthetic -- stay usable
without torch, e.g. from the python3.9 golden generator):
  constants  reference constants (envs.py)
  synthetic  seeded synthetic scenes
  _lib       ctypes binding of libsimaps.so (the C-ABI in include/simaps.h)
  batch      device-resident batched scene packing + the fused get_state launch, ingest, movement
             paths, reward lookups, raw-grid SSSP / paths
  vector_env drop-ins for VectorEnv.get_state (VectorEnvObservations) and GridGraph
  policy_input  device stacks -> DQNPolicy inputs (zero-copy CHW views, per-group batches)
  camera     the reference cameras' projection constants (ingest)
  reference_adapter  reads a reference VectorEnv into scene descriptors
"""
__all__ = ['constants', 'synthetic']
