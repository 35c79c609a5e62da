# Round-5: the pipelined large-grid SPFA pop (csrc/grid_large.h, SIMAPS_GL_PIPE) -- the large-grid
# and GridGraph tests, then the gridgraph_large row against the serial pop (libsimaps_glser.so,
# SIMAPS_GL_PIPE=0), alternating.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "300|r5l_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -v --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "200|r5l_large_pipe_1|python tools/bench_extra.py --gridgraph-large" \
  "200|r5l_large_ser_1|SIMAPS_LIB=$L/libsimaps_glser.so python tools/bench_extra.py --gridgraph-large" \
  "200|r5l_large_pipe_2|python tools/bench_extra.py --gridgraph-large" \
  "200|r5l_large_ser_2|SIMAPS_LIB=$L/libsimaps_glser.so python tools/bench_extra.py --gridgraph-large"
