# Round-5: every reference experiment config (93) against the oracle, then the whole -m gpu suite.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "400|r5o_pytest_refcfg|python -u -m pytest tests/test_gpu_reference_configs.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "600|r5o_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
