#!/bin/bash
# Compute-side counter passes (SQ / GRBM) of the ingest kernels (tools/bench_extra.py --ingest-only),
# GPU box.  tools/sq_profile_ingest.sh <tag> -> gpurun_out/sq_ingest_<tag>/pass{1,2,3}_counter_collection.csv
# Same passes as tools/sq_profile.sh: one rocprofv3 run each, no tracing, own hard time limit.
set -e
tag=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/sq_ingest_$tag
mkdir -p "$out"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$out" -o pass$i -- \
      python3 tools/bench_extra.py --ingest-only > "$out/bench_pass$i.json"
done
echo "sq profiles in $out"
