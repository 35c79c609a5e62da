#!/bin/bash
# A/B of the large-window fixpoint in one GPU call (round 6): the large-grid tests on the tree's
# library, then tools/bench_extra.py --gridgraph-large on it, on an older build
# (spatial-intention-maps_amd/simaps/libsimaps_gtfull.so, built from another revision, whose source hash
# the caller writes to tools/.ab_hash for SIMAPS_AB_SOURCE_HASH), and on the tree's library again.
# Run through tools/gpurun_retry.sh; delete both A/B files afterwards.  Logs: gpurun_out/<TAG>_{tests,new,old,new2}.*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6dl}
mkdir -p gpurun_out
H=$(cat tools/.ab_hash)
timeout -k 10 300 python -u -m pytest tests/test_gpu_gridgraph_large.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 &&
timeout -k 10 200 python tools/bench_extra.py --gridgraph-large > gpurun_out/${tag}_new.jsonl 2>&1 &&
SIMAPS_LIB=spatial-intention-maps_amd/simaps/libsimaps_gtfull.so SIMAPS_AB_SOURCE_HASH=$H timeout -k 10 200 python tools/bench_extra.py --gridgraph-large > gpurun_out/${tag}_old.jsonl 2>&1 &&
timeout -k 10 200 python tools/bench_extra.py --gridgraph-large > gpurun_out/${tag}_new2.jsonl 2>&1
