#!/bin/bash
# Kernel trace + HBM counter passes of the ingest kernels (tools/bench_extra.py --ingest-only), GPU box.
#   tools/profile_ingest.sh <tag>   -> gpurun_out/prof_<tag>_ingest/
set -e
tag=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}_ingest
mkdir -p "$out"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o ktrace -- \
    python3 tools/bench_extra.py --ingest-only > "$out/bench_ktrace.json"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out" -o pmc_fetch -- \
    python3 tools/bench_extra.py --ingest-only > "$out/bench_fetch.json"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out" -o pmc_write -- \
    python3 tools/bench_extra.py --ingest-only > "$out/bench_write.json"
echo "ingest profiles in $out"
