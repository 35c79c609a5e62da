# Round-4 final-build fuzz: get_state (15,616 fresh-seed stacks, perturbed poses, both rotate
# roundings), the 8(f) rows (28,672 paths + lookups), ingest (fresh frames).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r4o_fuzz_states|python tools/fuzz_states.py 256 16 --perturb" \
  "600|r4o_fuzz_states_plain|python tools/fuzz_states.py 256 16 --perturb --plain" \
  "600|r4o_fuzz_rows|python tools/fuzz_rows.py 256 4 16" \
  "300|r4o_fuzz_ingest|python tools/fuzz_ingest.py 16 16"
