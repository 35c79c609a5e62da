#!/bin/bash
# Ingest kernel A/B on the GPU box (tools/bench_extra.py --ingest-only: kernels alone), alternating
# twice.  Arguments: library file names under spatial-intention-maps_amd/simaps/ (default:
# libsimaps_base.so -- a build of another revision, e.g. tools/prod_build.sh <rev> base -- against
# the product libsimaps.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
libs="${@:-libsimaps_base.so libsimaps.so}"
for rep in 1 2; do
for lib in $libs; do
  SIMAPS_LIB=$PWD/spatial-intention-maps_amd/simaps/$lib timeout -k 10 120 python tools/bench_extra.py --ingest-only > gpurun_out/ing_$lib.$rep.log 2>&1 || exit 1
  grep '^{' gpurun_out/ing_$lib.$rep.log | python -c "import json,sys; d=json.load(sys.stdin); print('$lib', round(d['gpu_ms_per_launch']*1e3,1), 'us', round(d['roofline']['frac'],3))"
done
done
