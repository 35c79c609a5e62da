#!/bin/bash
# Kernel-trace + HBM counter profiles of the bench workload (run on the GPU box).
#   tools/profile_round.sh <tag> [bench args...]
# -> gpurun_out/prof_<tag>/{ktrace,pmc_fetch,pmc_write}_*.csv ; then, on the dev box,
#    python tools/collect_profiles.py <tag>  copies the summaries into profiles/.
# Counters are collected in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass),
# never together with runtime / sys tracing.
set -e
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
args="$* --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o ktrace -- \
    python3 bench.py --steps 30 --warmup 3 $args > "$out/bench_ktrace.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out" -o pmc_fetch -- \
    python3 bench.py --steps 5 --warmup 1 $args > "$out/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out" -o pmc_write -- \
    python3 bench.py --steps 5 --warmup 1 $args > "$out/bench_write.json"
echo "profiles in $out"
