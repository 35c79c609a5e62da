# Round-4 path pop v7 (double-buffered read-ahead issued before the common-pop test) as an A/B
# library against the tree's v6: all GPU tests through v7, per-pop stamps, path bench, A/B against
# the round-3 pop and v6, path fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4p_pytest_v7|SIMAPS_LIB=$P/libsimaps_prod_asmv7.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4p_pathbench_stamps_v7|SIMAPS_PROF_LIB=$P/libsimaps_prof_asmv7.so python tools/path_bench.py --stamps" \
  "200|r4p_pathbench_stamps_v6|python tools/path_bench.py --stamps" \
  "200|r4p_pathbench_v7|SIMAPS_LIB=$P/libsimaps_prod_asmv7.so python tools/path_bench.py" \
  "200|r4p_path_ab|for r in 1 2; do for l in prod_r3pop prod_asmv7; do SIMAPS_LIB=$P/libsimaps_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; done" \
  "300|r4p_rows_fuzz_v7|SIMAPS_LIB=$P/libsimaps_prod_asmv7.so python tools/fuzz_rows.py 128 4 16"
