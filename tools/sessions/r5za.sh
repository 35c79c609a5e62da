# Round-5: where a tiled large-grid pop spends its cycles (stats build: pops, tile misses, cycles
# per section), and the memory loop's pops / cycles for scale.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5za_stats|SIMAPS_LIB=$L/libsimaps_glstats.so python tools/debug/gl_pipe_stats.py"
