# Round-5 final check on the final tree: every -m gpu test, smoke(), the bench line.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r5zb_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5zb_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r5zb_bench|python bench.py"
