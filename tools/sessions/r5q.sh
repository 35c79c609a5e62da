# Round-5: the timed region's clock stops before the closing barrier -- the driver's command form
# (20 steps, 5 warmup) at N = 1, on one RCCL rank (--init-dist), and two self-spawned ranks sharing the GPU.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "200|r5q_bench_n1|python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r5q_rccl_1rank|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --init-dist --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r5q_bench_n1_b|python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r5q_rccl_1rank_b|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --init-dist --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r5q_spawn2|python bench.py --gpus 2 --shared-gpu --steps 20 --warmup 5 --no-cpu-baseline"
