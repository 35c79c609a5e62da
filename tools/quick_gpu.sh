#!/bin/bash
# One GPU iteration: parity tests, a short bench line, the per-phase stamp profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_bench.log 2>&1 || { tail -20 gpurun_out/q_bench.log; exit 1; }
grep metric gpurun_out/q_bench.log
timeout -k 10 120 python tools/phase_profile.py ${PH_ARGS:-} > gpurun_out/q_ph.log 2>&1 || { tail -20 gpurun_out/q_ph.log; exit 1; }
grep -v amdgpu.ids gpurun_out/q_ph.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, v) for k, v in d.items()]"
