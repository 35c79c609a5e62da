# Round-4 path pop v3 (wrap budget, derived count): parity, per-pop stamps, A/B against the round-3
# pop and asm v2, fresh-seed path fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4k_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200|r4k_pathbench_stamps|python tools/path_bench.py --stamps" \
  "200|r4k_pathbench|python tools/path_bench.py" \
  "200|r4k_path_ab|for r in 1 2; do for l in r3pop asmv2; do SIMAPS_LIB=$P/libsimaps_prod_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; done" \
  "500|r4k_rows_fuzz|python tools/fuzz_rows.py 64 4 16"
