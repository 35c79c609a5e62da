# Round-4 path pop: parity (all GPU tests), per-pop timing (stamp build), A/B of the round-3 pop /
# the C++ pipelined pop / the asm pop, and a fresh-seed path fuzz on the product build.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4j_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4j_pathbench_stamps|python tools/path_bench.py --stamps" \
  "200|r4j_pathbench|python tools/path_bench.py" \
  "200|r4j_path_ab|for l in r3pop cpipe; do SIMAPS_LIB=$P/libsimaps_prod_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; for l in r3pop cpipe; do SIMAPS_LIB=$P/libsimaps_prod_\$l.so python tools/path_ab.py; done; python tools/path_ab.py" \
  "500|r4j_rows_fuzz|python tools/fuzz_rows.py 64 4 16"
