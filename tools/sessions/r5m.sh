# Round-5: why the pipelined large-grid pop is slower -- pops, fast / slow pops and cycles of one
# 500 x 500 path under stats builds of both pops.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5m_stats_pipe|SIMAPS_LIB=$L/libsimaps_glstats.so python tools/debug/gl_pipe_stats.py" \
  "120|r5m_stats_ser|SIMAPS_LIB=$L/libsimaps_glstats_ser.so python tools/debug/gl_pipe_stats.py"
