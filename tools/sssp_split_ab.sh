#!/bin/bash
# Split-sweep SSSP A/B on the GPU box (tools/sssp_split_ab.py): each variant build
# (tools/prod_build.sh WT <name> -DSIMAPS_SSSP_SPLIT_L=.. -DSIMAPS_SSSP_SPLIT_S=..) passes the SSSP
# parity tests, then the variants are timed alternately, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
libs="${@:-base l2s1 l2s2 l3s1 l4s2}"
for v in $libs; do
  SIMAPS_LIB=$PWD/spatial-intention-maps_amd/simaps/libsimaps_prod_$v.so timeout -k 10 200 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "room_width_92 or sssp_grid or sp_distance or gridgraph_dropin or distance_to_receptacle" \
    > gpurun_out/split_test_$v.log 2>&1 || { echo "tests failed: $v"; tail -5 gpurun_out/split_test_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/split_test_$v.log)"
done
for rep in 1 2; do
  for v in $libs; do
    SIMAPS_LIB=$PWD/spatial-intention-maps_amd/simaps/libsimaps_prod_$v.so timeout -k 10 200 python tools/sssp_split_ab.py \
      > gpurun_out/split_ab_$v.$rep.log 2>&1 || exit 1
    grep '^{' gpurun_out/split_ab_$v.$rep.log
  done
done
