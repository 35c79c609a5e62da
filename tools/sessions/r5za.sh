# Round-5: the LDS-tiled large-grid SPFA as an A/B build (SIMAPS_GL_LDS=1: libsimaps_gltile.so)
# against the product's memory loop -- a stats build (pops, tile misses, cycles per section), the
# gridgraph_large row alternating, and the large-grid tests on the tiled build and on its 64-entry-
# ring hand-over variant (libsimaps_glq64.so).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5za_stats|SIMAPS_LIB=$L/libsimaps_glstats.so python tools/debug/gl_pipe_stats.py" \
  "200|r5za_large_tile|SIMAPS_LIB=$L/libsimaps_gltile.so python tools/bench_extra.py --gridgraph-large" \
  "200|r5za_large_mem|python tools/bench_extra.py --gridgraph-large" \
  "300|r5za_pytest_large_tile|SIMAPS_LIB=$L/libsimaps_gltile.so python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "300|r5za_pytest_large_q64|SIMAPS_LIB=$L/libsimaps_glq64.so python -u -m pytest tests/test_gpu_gridgraph_large.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'large or gridgraph'" \
  "300|r5za_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -m gpu -x -q --timeout 120 --timeout-method thread"
