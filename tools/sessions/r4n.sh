# Round-4 final-build profiles: get_state kernel trace + FETCH / WRITE_SIZE passes of the bench
# workload, the per-phase stamps (roofline.binding), the BASELINE configs, the RCCL 1-rank line.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "600|r4n_prof|bash tools/profile_round.sh r4n" \
  "120|r4n_ph|python tools/phase_profile.py" \
  "400|r4n_configs|bash tools/bench_configs.sh" \
  "200|r4n_rccl|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --init-dist --steps 50 --no-cpu-baseline"
