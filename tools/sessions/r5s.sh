# Round-5: the timed region's cost with and without the bench's timing events, and the bench line
# itself at the driver's 20 / 5 steps, in one call (one box).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200|r5s_fixed|python tools/debug/fixed_overhead.py" \
  "200|r5s_bench20|python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r5s_bench200|python bench.py --gpus 1 --no-cpu-baseline" \
  "200|r5s_fixed_b|python tools/debug/fixed_overhead.py" \
  "200|r5s_bench20_b|python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
