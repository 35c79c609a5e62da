# Round-5: the fixed cost of a timed region (K = 0 ... 200), default vs spin-wait synchronisation.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200|r5r_fixed_default|python tools/debug/fixed_overhead.py" \
  "200|r5r_fixed_spin|python tools/debug/fixed_overhead.py --spin" \
  "200|r5r_fixed_default_b|python tools/debug/fixed_overhead.py" \
  "200|r5r_fixed_spin_b|python tools/debug/fixed_overhead.py --spin"
