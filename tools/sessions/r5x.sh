# Round-5: which instruction-cache / fetch counters gfx950 exposes (rocprofv3 --list-avail).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r5x_list_avail.txt 2>&1
echo "rc=$?"
grep -i -E "ICACHE|IFETCH|SQC_|INST_" gpurun_out/r5x_list_avail.txt | head -80 > gpurun_out/r5x_icache_counters.txt || true
wc -l gpurun_out/r5x_list_avail.txt
