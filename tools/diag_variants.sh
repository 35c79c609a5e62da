#!/bin/bash
# Phase-stamp profile of each diagnostic variant build given as arguments (libsimaps_<NAME>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "$@"; do
  SIMAPS_PROF_LIB=spatial-intention-maps_amd/simaps/libsimaps_$n.so timeout -k 10 120 python tools/phase_profile.py ${PH_ARGS:-} > gpurun_out/v_$n.log 2>&1 || { tail -20 gpurun_out/v_$n.log; exit 1; }
  echo "== $n"
  grep -v amdgpu.ids gpurun_out/v_$n.log | python -c "import json,sys; d=json.load(sys.stdin); [print(' ', k, v) for k, v in d.items() if k in ('total_us_median','spread_us')]"
done
