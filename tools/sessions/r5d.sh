# Round-5: the large-window GridGraph after the DPP fix (r5c: a select around the DPP neighbour
# exchange became a branch, and the disabled lane read as 0) and the register-tracked SPFA front:
# the debug diff, the large-grid GPU tests, the bench row.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "120|r5d_gl_diff|python tools/debug/gl_sssp_diff.py" \
  "400|r5d_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 300 --timeout-method thread" \
  "200|r5d_extra_large|python tools/bench_extra.py --gridgraph-large"
