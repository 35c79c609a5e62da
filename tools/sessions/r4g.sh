cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "400|r4g_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|r4g_extra|python tools/bench_extra.py" \
  "200|r4g_envstep|python tools/bench_extra.py --env-step" \
  "200|r4g_envstep_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_prof -o envstep -- python tools/bench_extra.py --env-step"
