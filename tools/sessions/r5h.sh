# Round-5: the product large-window build (1 wave per direction, 32 lines prefetched) through the
# large-grid tests and its bench row; the no-drain SPFA pop variant (timing + the same tests).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "400|r5h_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 300 --timeout-method thread" \
  "200|r5h_extra_large|python tools/bench_extra.py --gridgraph-large" \
  "400|r5h_pytest_large_nodrain|SIMAPS_LIB=$L/libsimaps_glnodrain.so python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 300 --timeout-method thread" \
  "200|r5h_extra_large_nodrain|SIMAPS_LIB=$L/libsimaps_glnodrain.so python tools/bench_extra.py --gridgraph-large"
