# Round-5 closing evidence on the final tree: every -m gpu test, smoke(), the bench line (default
# twice, and the driver's 20 / 5 form), the kernel trace + FETCH/WRITE passes, every BASELINE
# config, the 8(f) rows, env step, mixed launch and large-grid rows, the self-spawned 2-rank
# rehearsal and the RCCL 1-rank line (clock now stops before the closing barrier), and a get_state
# fuzz on fresh seeds.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r5u_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r5u_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r5u_bench|python bench.py" \
  "300|r5u_bench2|python bench.py" \
  "200|r5u_bench20|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "600|r5u_prof|bash tools/profile_round.sh r5u" \
  "400|r5u_configs|bash tools/bench_configs.sh" \
  "400|r5u_extra|python tools/bench_extra.py" \
  "200|r5u_env|python tools/bench_extra.py --env-step" \
  "200|r5u_mixed|python tools/bench_extra.py --mixed" \
  "200|r5u_large|python tools/bench_extra.py --gridgraph-large" \
  "200|r5u_spawn2|python bench.py --gpus 2 --shared-gpu --steps 100 --warmup 10" \
  "200|r5u_rccl|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --init-dist --steps 50 --no-cpu-baseline" \
  "600|r5u_fuzz_states|SIMAPS_FUZZ_SEED0=30000 python tools/fuzz_states.py 256 16 --perturb"
