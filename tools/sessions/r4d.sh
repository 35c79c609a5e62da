cd "${GRAFT_REPO_ROOT}"
P=spatial-intention-maps_amd/simaps
SIMAPS_LIB=$P/libsimaps_prod_check.so timeout -k 10 120 python tools/sssp_debug.py > gpurun_out/r4d_dbg_check.log 2>&1 || { tail -5 gpurun_out/r4d_dbg_check.log; exit 1; }
tail -1 gpurun_out/r4d_dbg_check.log
timeout -k 10 120 python tools/phase_profile.py > gpurun_out/r4d_ph_check.log 2>&1 || exit 1
timeout -k 10 200 bash tools/ab_bench.sh marks check
