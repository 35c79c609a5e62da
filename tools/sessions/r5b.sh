# Round-5: GridGraph beyond the LDS window (csrc/grid_large.h): its GPU tests and bench row; then the
# latency accounting of the path kernels (stamp build) and the raw per-workgroup stamps of get_state
# (the tail model), and each agent rendered alone.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "300|r5b_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 240 --timeout-method thread" \
  "200|r5b_extra_large|python tools/bench_extra.py --gridgraph-large" \
  "200|r5b_path_latency|python tools/path_bench.py --stamps --latency" \
  "200|r5b_phase|python tools/phase_profile.py --dump gpurun_out/r5b_stamps.npy" \
  "200|r5b_agent_times|python tools/agent_times.py lifting_4-small_divider 64"
