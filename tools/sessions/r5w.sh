# Round-5: parity fuzz at scale on fresh seeds with the remaining GPU time -- paths and lookups in
# the compact and early-exit modes (the automatic and overlapped modes ran in r5k / r5n), get_state
# through the mixed launch in the CHW layout's fuzz form (hwc views), and ingest.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r5w_fuzz_rows_compact|python tools/fuzz_rows.py --path-mode 1 --seed0 40000 256 4 16" \
  "600|r5w_fuzz_rows_early|python tools/fuzz_rows.py --path-mode 2 --seed0 41000 256 4 16" \
  "600|r5w_fuzz_ingest|SIMAPS_FUZZ_SEED0=42000 python tools/fuzz_ingest.py 512 16" \
  "900|r5w_fuzz_mixed|SIMAPS_FUZZ_SEED0=43000 python tools/fuzz_states.py 1024 16 --perturb --mixed"
