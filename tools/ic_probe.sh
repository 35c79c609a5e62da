# Per-dispatch SQ counters of one agent's workgroup (tools/one_agent.py), product vs a variant lib.
set -e
export TMPDIR=/tmp
for lib in libsimaps.so libsimaps_v2.so; do
  for P in "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    SIMAPS_LIB=spatial-intention-maps_amd/simaps/$lib timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/one_$lib -o pmc -- python3 tools/one_agent.py lifting_4-large_rooms 16 4 5
  done
done
