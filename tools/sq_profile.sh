#!/bin/bash
# Compute-side counter passes (SQ / GRBM) of get_state_kernel on the bench workload (GPU box).
#   tools/sq_profile.sh <tag> [bench args...]
# -> gpurun_out/sq_<tag>/pass{1,2,3}_counter_collection.csv ; summarised by tools/sq_summary.py.
# One rocprofv3 run per pass (<= 8 SQ + 2 GRBM counters each), kernel trace off, never combined
# with runtime / sys tracing; each pass under its own hard time limit.
set -e
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/sq_$tag
mkdir -p "$out"
args="--steps 5 --warmup 1 --no-cpu-baseline $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$out" -o pass$i -- \
      python3 bench.py $args > "$out/bench_pass$i.json"
done
echo "sq profiles in $out"
