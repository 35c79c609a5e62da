#!/bin/bash
# Kernel-only ingest timing of each libsimaps_ing_<NAME>.so variant (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in "$@"; do
  SIMAPS_LIB=$PWD/spatial-intention-maps_amd/simaps/libsimaps_ing_$n.so timeout -k 10 120 python tools/bench_extra.py --ingest-only > gpurun_out/ing_$n.log 2>&1 || { tail -5 gpurun_out/ing_$n.log; exit 1; }
  grep '^{' gpurun_out/ing_$n.log | python -c "import json,sys; d=json.load(sys.stdin); print('$n', round(d['gpu_ms_per_launch']*1e3,1), 'us', round(d['roofline']['frac'],3))"
done
