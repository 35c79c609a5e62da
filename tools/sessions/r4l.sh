# Round-4 path pop v4 (one budget, no per-pop state) and v5 (v4 unrolled by two) as A/B libraries
# against the tree's v3: all GPU tests through each, per-pop stamps, path bench, A/B with the
# round-3 pop, fresh-seed path fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4l_pytest_v5|SIMAPS_LIB=$P/libsimaps_prod_asmv5.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "420|r4l_pytest_v4|SIMAPS_LIB=$P/libsimaps_prod_asmv4.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4l_pathbench_stamps_v5|SIMAPS_PROF_LIB=$P/libsimaps_prof_asmv5.so python tools/path_bench.py --stamps" \
  "200|r4l_pathbench_stamps_v4|SIMAPS_PROF_LIB=$P/libsimaps_prof_asmv4.so python tools/path_bench.py --stamps" \
  "200|r4l_pathbench_v5|SIMAPS_LIB=$P/libsimaps_prod_asmv5.so python tools/path_bench.py" \
  "200|r4l_path_ab|for r in 1 2; do for l in prod_r3pop prod_asmv4 prod_asmv5; do SIMAPS_LIB=$P/libsimaps_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; done" \
  "300|r4l_rows_fuzz_v5|SIMAPS_LIB=$P/libsimaps_prod_asmv5.so python tools/fuzz_rows.py 64 4 16" \
  "300|r4l_rows_fuzz_v4|SIMAPS_LIB=$P/libsimaps_prod_asmv4.so python tools/fuzz_rows.py 64 4 16"
