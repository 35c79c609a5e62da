# Round-5: every reference experiment config: states, then movement paths and reward lookups, vs the oracle.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r5p_pytest_refcfg|python -u -m pytest tests/test_gpu_reference_configs.py -m gpu -q --timeout 120 --timeout-method thread"
