cd "${GRAFT_REPO_ROOT}"
P=spatial-intention-maps_amd/simaps
for v in marks check both; do
  SIMAPS_LIB=$P/libsimaps_prod_$v.so timeout -k 10 120 python tools/sssp_debug.py > gpurun_out/r4c_dbg_$v.log 2>&1 || { tail -5 gpurun_out/r4c_dbg_$v.log; exit 1; }
  tail -1 gpurun_out/r4c_dbg_$v.log
done
