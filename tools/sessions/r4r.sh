# Round-4 closing check on the committed tree: all GPU tests, smoke, the headline bench twice.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "420|r4r_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r4r_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r4r_bench|python bench.py" \
  "300|r4r_bench2|python bench.py"
