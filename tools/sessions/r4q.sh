# Round-4 A/B: snap + SSSP start under one group barrier on the sweep track ("fuse") against HEAD:
# all GPU tests through the fused build, bench A/B on the BASELINE line and two other configs,
# per-phase stamps of both, get_state fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4q_pytest_fuse|SIMAPS_LIB=$P/libsimaps_prod_fuse.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|r4q_ab_base|bash tools/ab_bench.sh head fuse" \
  "300|r4q_ab_push|BENCH_ARGS='--config pushing_4-large_empty --envs 256' bash tools/ab_bench.sh head fuse" \
  "300|r4q_ab_rescue|BENCH_ARGS='--config rescue_4-small_empty --total-envs 2048' bash tools/ab_bench.sh head fuse" \
  "120|r4q_ph_head|python tools/phase_profile.py" \
  "120|r4q_ph_fuse|SIMAPS_PROF_LIB=$P/libsimaps_prof_fuse.so python tools/phase_profile.py" \
  "600|r4q_fuzz_states_fuse|SIMAPS_LIB=$P/libsimaps_prod_fuse.so python tools/fuzz_states.py 128 16 --perturb"
