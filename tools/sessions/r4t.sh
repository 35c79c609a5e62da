# Round-4 fresh-seed path fuzz of the path modes on the final tree: mode 3 forced at 2,048 paths per
# launch (several workgroup waves), and the automatic mode on both sides of its switch (256 paths per
# launch: overlapped; 2,048: sequential early exit).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "300|r4t_fuzz_ovl|python tools/fuzz_rows.py --path-mode 3 --seed0 9000 128 4 16" \
  "300|r4t_fuzz_auto_small|python tools/fuzz_rows.py --path-mode 0 --seed0 9500 16 4 16" \
  "300|r4t_fuzz_auto_large|python tools/fuzz_rows.py --path-mode 0 --seed0 9700 128 4 16"
