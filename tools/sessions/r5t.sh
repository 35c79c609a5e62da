# Round-5: per-step time of a cold vs a heated GPU (fresh processes), twice.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200|r5t_warm_1|python tools/debug/warm_probe.py --heat 300" \
  "200|r5t_warm_2|python tools/debug/warm_probe.py --heat 300" \
  "200|r5t_warm_3|python tools/debug/warm_probe.py --heat 50"
