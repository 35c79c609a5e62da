# Round-5: the mixed batch's array fast path and the other new GPU tests, then a larger parity fuzz
# on fresh seeds: get_state 1,024 envs per configuration in each rotate rounding (seeds past every
# earlier run's), the mixed launch over 512 envs per configuration, paths / lookups in the
# overlapped path mode, and ingest.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "300|r5n_pytest_mixed|python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_gridgraph_large.py -m gpu -x -v --timeout 120 --timeout-method thread" \
  "900|r5n_fuzz_states|SIMAPS_FUZZ_SEED0=20000 python tools/fuzz_states.py 1024 16 --perturb" \
  "900|r5n_fuzz_states_plain|SIMAPS_FUZZ_SEED0=20000 python tools/fuzz_states.py 1024 16 --perturb --plain" \
  "900|r5n_fuzz_mixed|SIMAPS_FUZZ_SEED0=22000 python tools/fuzz_states.py 512 16 --perturb --mixed" \
  "600|r5n_fuzz_rows_ovl|python tools/fuzz_rows.py --path-mode 3 --seed0 16000 256 4 16" \
  "600|r5n_fuzz_ingest|SIMAPS_FUZZ_SEED0=24000 python tools/fuzz_ingest.py 128 16"
