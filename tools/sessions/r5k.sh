# Round-5 evidence on the tree with the mixed-configuration launch (the get_state kernel gained the
# intention-channel robot-count check): every -m gpu test, smoke(), the bench line (twice), the
# get_state kernel trace + FETCH/WRITE passes and the stamp profile, every BASELINE config, the 8(f)
# rows and env step, the mixed launch timing, and the fuzz: get_state in both roundings, through
# the mixed launch, and fresh-seed paths.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "420|r5k_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5k_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r5k_bench|python bench.py" \
  "300|r5k_bench2|python bench.py" \
  "600|r5k_prof|bash tools/profile_round.sh r5k" \
  "120|r5k_phase|python tools/phase_profile.py --dump gpurun_out/r5k_stamps.npy" \
  "400|r5k_configs|bash tools/bench_configs.sh" \
  "400|r5k_extra|python tools/bench_extra.py" \
  "200|r5k_env|python tools/bench_extra.py --env-step" \
  "200|r5k_mixed|python tools/bench_extra.py --mixed" \
  "600|r5k_fuzz_mixed|python tools/fuzz_states.py 128 16 --perturb --mixed" \
  "600|r5k_fuzz_states|python tools/fuzz_states.py 256 16 --perturb" \
  "600|r5k_fuzz_states_plain|python tools/fuzz_states.py 256 16 --perturb --plain" \
  "400|r5k_fuzz_rows|python tools/fuzz_rows.py --path-mode 0 --seed0 14000 128 4 16"
