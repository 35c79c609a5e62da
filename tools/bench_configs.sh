#!/bin/bash
# Bench lines of every BASELINE config on one GPU (same kernel), at the BASELINE launch sizes:
# configs[0] lifting_1-small_empty (256 envs x 1), [1] lifting_4-small_divider (64 x 4),
# [2] pushing_4-large_empty (256 x 4), [3] lifting_2_throwing_2-large_empty (1024 x 4, strong mode:
# the whole job on this GPU), [4] rescue_4-small_empty (2048 x 4, strong mode).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "lifting_1-small_empty --envs 256" "pushing_4-large_empty --envs 256" "lifting_2_throwing_2-large_empty --total-envs 1024" "rescue_4-small_empty --total-envs 2048" "lifting_4-small_divider --envs 64"; do
  set -- $spec
  timeout -k 10 180 python bench.py --config $spec --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/cfg_$1.log 2>&1 || { tail -5 gpurun_out/cfg_$1.log; exit 1; }
  grep '^{' gpurun_out/cfg_$1.log | tail -1 | tee -a gpurun_out/bench_configs.jsonl | python -c "import json,sys; d=json.load(sys.stdin); print('$1', d['config']['stacks_per_step'], round(d['value']/1e6, 3), 'M stacks/s', round(d['roofline']['frac'], 3), round(d['ms_per_step']*1e3, 1), 'us/step')"
done
