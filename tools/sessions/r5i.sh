# Round-5: the asm SPFA pop without lane 8's two selects (two VALU fewer per pop) -- the path tests,
# a fresh-seed path fuzz, and an A/B against the previous revision (libsimaps_prev.so /
# libsimaps_prevprof.so, built from HEAD before the change): launch times, ns per pop, env step.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "300|r5i_pytest_paths|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'path or spfa or overlap or gridgraph or ring or fault'" \
  "400|r5i_fuzz_rows|python tools/fuzz_rows.py --path-mode 0 --seed0 13000 128 4 16" \
  "300|r5i_fuzz_rows_m2|python tools/fuzz_rows.py --path-mode 2 --seed0 13500 128 4 16" \
  "150|r5i_lat_new_1|python tools/path_bench.py --latency" \
  "150|r5i_lat_prev_1|SIMAPS_LIB=$L/libsimaps_prev.so python tools/path_bench.py --latency" \
  "150|r5i_lat_new_2|python tools/path_bench.py --latency" \
  "150|r5i_lat_prev_2|SIMAPS_LIB=$L/libsimaps_prev.so python tools/path_bench.py --latency" \
  "150|r5i_st_new|python tools/path_bench.py --stamps --latency" \
  "150|r5i_st_prev|SIMAPS_PROF_LIB=$L/libsimaps_prevprof.so python tools/path_bench.py --stamps --latency" \
  "200|r5i_env_new|python tools/bench_extra.py --env-step" \
  "200|r5i_env_prev|SIMAPS_LIB=$L/libsimaps_prev.so python tools/bench_extra.py --env-step"
