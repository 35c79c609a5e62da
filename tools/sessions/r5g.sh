# Round-5 closing session on the final tree: every -m gpu test, smoke(), the BASELINE bench line
# (twice), the self-spawned 2-rank rehearsal and the RCCL 1-rank line; the get_state kernel trace +
# FETCH/WRITE passes (profiles/pmc_traffic.json) and stamp profile; every BASELINE config; the 8(f)
# rows (incl. the env step under a kernel trace and the large-grid GridGraph); the path latency
# accounting; the get_state fuzz (15,616 stacks, both roundings) and a fresh-seed path fuzz.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "420|r5g_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5g_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r5g_bench|python bench.py" \
  "300|r5g_bench2|python bench.py" \
  "200|r5g_spawn2|python bench.py --gpus 2 --shared-gpu --steps 100 --warmup 10" \
  "200|r5g_rccl|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --init-dist --steps 50 --no-cpu-baseline" \
  "600|r5g_prof|bash tools/profile_round.sh r5g" \
  "120|r5g_phase|python tools/phase_profile.py --dump gpurun_out/r5g_stamps.npy" \
  "400|r5g_configs|bash tools/bench_configs.sh" \
  "400|r5g_extra|python tools/bench_extra.py" \
  "200|r5g_envstep_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_prof_env -o envstep -- python tools/bench_extra.py --env-step" \
  "200|r5g_extra_large|python tools/bench_extra.py --gridgraph-large" \
  "200|r5g_path_latency|python tools/path_bench.py --stamps --latency" \
  "600|r5g_fuzz_states|python tools/fuzz_states.py 256 16 --perturb" \
  "600|r5g_fuzz_states_plain|python tools/fuzz_states.py 256 16 --perturb --plain" \
  "400|r5g_fuzz_rows|python tools/fuzz_rows.py --path-mode 0 --seed0 12000 128 4 16"
