cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "420|r4i_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4i_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r4i_bench|python bench.py" \
  "120|r4i_ph|python tools/phase_profile.py"
