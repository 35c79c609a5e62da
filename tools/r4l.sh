# Round-4 path pop v4 (one budget, no per-pop state) as an A/B library against the tree's v3:
# all GPU tests through v4, per-pop stamps, A/B with the round-3 pop, fresh-seed path fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4l_pytest_v4|SIMAPS_LIB=$P/libsimaps_prod_asmv4.so python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4l_pathbench_stamps|SIMAPS_PROF_LIB=$P/libsimaps_prof_asmv4.so python tools/path_bench.py --stamps" \
  "200|r4l_pathbench|SIMAPS_LIB=$P/libsimaps_prod_asmv4.so python tools/path_bench.py" \
  "200|r4l_path_ab|for r in 1 2; do for l in prod_r3pop prod_asmv4; do SIMAPS_LIB=$P/libsimaps_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; done" \
  "500|r4l_rows_fuzz|SIMAPS_LIB=$P/libsimaps_prod_asmv4.so python tools/fuzz_rows.py 64 4 16"
