#!/bin/bash
# Bench A/B of product builds spatial-intention-maps_amd/simaps/libsimaps_prod_<name>.so in one GPU call:
#   [BENCH_ARGS="--config X --envs E"] [AB_OLD_ABI=n] tools/ab_bench.sh NAME1 NAME2 ...   (two rounds, alternating)
# AB_OLD_ABI: also accept builds of an older revision with ABI version n (get_state's signature unchanged)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2; do for v in "$@"; do
  SIMAPS_AB_OLD_ABI=${AB_OLD_ABI:-} SIMAPS_LIB=spatial-intention-maps_amd/simaps/libsimaps_prod_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${v}_${i}.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_${i}.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${v}_${i}.log)"
done; done
