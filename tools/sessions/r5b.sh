# Round-5: GridGraph beyond the LDS window (csrc/grid_large.h): its GPU tests, then its bench row.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "300|r5b_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 240 --timeout-method thread" \
  "200|r5b_extra_large|python tools/bench_extra.py --gridgraph-large"
