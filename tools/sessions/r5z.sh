# Round-5: the large-grid SPFA on LDS tiles (csrc/grid_large.h gl_spfa_lds) -- the large-grid and
# GridGraph tests on the product build and on a build whose 64-entry queue ring hands over to the
# memory loop mid-run (libsimaps_glq64.so), then the gridgraph_large row against the memory loop
# alone (libsimaps_glmem.so, SIMAPS_GL_LDS=0), alternating.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "300|r5z_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "300|r5z_pytest_large_q64|SIMAPS_LIB=$L/libsimaps_glq64.so python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "200|r5z_large_lds_1|python tools/bench_extra.py --gridgraph-large" \
  "200|r5z_large_mem_1|SIMAPS_LIB=$L/libsimaps_glmem.so python tools/bench_extra.py --gridgraph-large" \
  "200|r5z_large_lds_2|python tools/bench_extra.py --gridgraph-large" \
  "200|r5z_large_mem_2|SIMAPS_LIB=$L/libsimaps_glmem.so python tools/bench_extra.py --gridgraph-large"
