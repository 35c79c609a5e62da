#!/bin/bash
# One rocprofv3 --pmc pass of the bench workload (own run, no tracing).  GPU box only.
#   tools/pmc_pass.sh <outdir> "<counters>" [bench args...]
set -e
out=$1; cnt=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 90 rocprofv3 --pmc $cnt --output-format csv -d "$out" -o pmc -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > "$out/bench.json"
