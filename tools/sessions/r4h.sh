cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "300|r4h_pytest|python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'receptacle or sp_distance or distance_to'" \
  "200|r4h_ab|AB_OLD_ABI=6 bash tools/ab_bench.sh base wt" \
  "120|r4h_ph|python tools/phase_profile.py" \
  "120|r4h_launch|python tools/launch_overhead.py" \
  "300|r4h_extra|python tools/bench_extra.py" \
  "200|r4h_envstep_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_prof -o envstep -- python tools/bench_extra.py --env-step"
