# Round-5: does instruction fetch stall get_state_kernel (198 KB of code)?  Instruction-cache and
# fetch counters of the bench workload, two SQC counters per pass (their block limit is not in
# the guide), each pass its own run under a hard limit; then the wave-cycle split for scale.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "100|r5y_ic1|bash tools/pmc_pass.sh gpurun_out/r5y_ic1 'SQC_ICACHE_REQ SQC_ICACHE_HITS'" \
  "100|r5y_ic2|bash tools/pmc_pass.sh gpurun_out/r5y_ic2 'SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE'" \
  "100|r5y_ic3|bash tools/pmc_pass.sh gpurun_out/r5y_ic3 'SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES'" \
  "100|r5y_if|bash tools/pmc_pass.sh gpurun_out/r5y_if 'SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE'"
