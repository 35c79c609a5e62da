# Round-5: the mixed-configuration launch (simaps_get_state_mixed) -- its tests first, then every
# -m gpu test, smoke(), the bench line (the get_state kernel gained the intention-channel robot-count
# check), every BASELINE config and the mixed vs per-configuration timing.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200|r5j_pytest_mixed|python -u -m pytest tests/test_gpu_mixed.py -m gpu -x -v --timeout 120 --timeout-method thread" \
  "420|r5j_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5j_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r5j_bench|python bench.py" \
  "200|r5j_mixed|python tools/bench_extra.py --mixed" \
  "400|r5j_configs|bash tools/bench_configs.sh"
