#!/bin/bash
# One GPU iteration: parity tests, a short bench line, the per-phase stamp profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q_bench.log 2>&1 || { tail -20 gpurun_out/q_bench.log; exit 1; }
grep metric gpurun_out/q_bench.log
timeout -k 10 120 python tools/phase_profile.py ${PH_ARGS:-} > gpurun_out/q_ph.log 2>&1 || { tail -20 gpurun_out/q_ph.log; exit 1; }
grep -v amdgpu.ids gpurun_out/q_ph.log | python -c "import json,sys; d=json.load(sys.stdin); print('total', d['total_us_median'], 'span', d['span_us'], d['split_groups_us'], d['pre_split_us'], d['distance_us'], d['rounds'], d['sweep_rounds_us'], d['first_sweep_us'], d['wave_sweep_r0_us'], d['render_front_us'], {k:v['median'] for k,v in d['phases_us'].items()})"
