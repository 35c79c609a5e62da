# Round-5: where a tiled large-grid pop spends its cycles (stats build: pops, tile misses, cycles
# per section), then the tiled product (the one-read tag lookup) against the memory loop, and the
# large-grid tests on the product and on the 64-entry-ring hand-over build.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5za_stats|SIMAPS_LIB=$L/libsimaps_glstats.so python tools/debug/gl_pipe_stats.py" \
  "200|r5za_large_lds|python tools/bench_extra.py --gridgraph-large" \
  "200|r5za_large_mem|SIMAPS_LIB=$L/libsimaps_glmem.so python tools/bench_extra.py --gridgraph-large" \
  "300|r5za_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "300|r5za_pytest_large_q64|SIMAPS_LIB=$L/libsimaps_glq64.so python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'"
