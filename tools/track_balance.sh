#!/bin/bash
# Sweep / render track ends (stamp build) for every BASELINE config (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "lifting_4-small_divider 64" "lifting_1-small_empty 256" "pushing_4-large_empty 256" "lifting_2_throwing_2-large_empty 256" "rescue_4-small_empty 256" "lifting_4-large_rooms 64"; do
  set -- $spec
  timeout -k 10 120 python tools/phase_profile.py --config $1 --envs $2 > gpurun_out/tb_$1.log 2>&1 || { tail -5 gpurun_out/tb_$1.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/tb_$1.log | python -c "
import json,sys; d=json.load(sys.stdin)
print('$1', 'total', d['total_us_median'], 'sweep_end', d['sweep_track_us']['end'], 'rounds', d['sweep_track_us']['rounds'], 'render_end', d['render_track_us']['end'], 'join', d['join_us'], 'dist', d['distance_us']['all'], 'rounds_n', d['rounds'])
print('   render', {k: v for k, v in d['render_track_us'].items()})"
done
