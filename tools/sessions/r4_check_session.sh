#!/bin/bash
# Round-4 GPU session: parity of the fixpoint-check SSSP build, bench A/B against the round-3
# inline-mark schedule (both product builds of the same tree), per-phase stamps of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|${TAG}_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|${TAG}_ab_base|bash tools/ab_bench.sh marks check" \
  "300|${TAG}_ab_push|BENCH_ARGS='--config pushing_4-large_empty --envs 256' bash tools/ab_bench.sh marks check" \
  "300|${TAG}_ab_lrooms|BENCH_ARGS='--config lifting_4-large_rooms --envs 64' bash tools/ab_bench.sh marks check" \
  "120|${TAG}_ph_check|python tools/phase_profile.py" \
  "120|${TAG}_ph_marks|SIMAPS_PROF_LIB=$P/libsimaps_profmarks.so python tools/phase_profile.py"
