# Round-5: the large-window sweeps with plain L1 loads + a per-round L1 invalidate: correctness (the
# large-grid tests + diff) and the bench row at 16 (product) / 8 / 32 lines prefetched.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5e_gl_diff|python tools/debug/gl_sssp_diff.py" \
  "400|r5e_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 300 --timeout-method thread" \
  "200|r5e_extra_large|python tools/bench_extra.py --gridgraph-large" \
  "200|r5e_extra_large_pf8|SIMAPS_LIB=$L/libsimaps_glpf8.so python tools/bench_extra.py --gridgraph-large" \
  "200|r5e_extra_large_pf32|SIMAPS_LIB=$L/libsimaps_glpf32.so python tools/bench_extra.py --gridgraph-large"
