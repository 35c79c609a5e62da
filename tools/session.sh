#!/bin/bash
# One parameterised GPU session (replaces the per-session scripts of rounds 4-5): named steps run in
# order through tools/gpu_session.sh, each under its own time limit, logs in gpurun_out/<TAG>_<step>.log;
# a timeout / abort / kill ends the session (no further GPU step).
#
#   gpurun --timeout 1200 -- bash tools/session.sh TAG step [step ...]
#
# Steps (extra arguments after '=' are appended to the step's command, e.g. fuzz_rows=--path-mode=4):
#   pytest smoke bench bench20 prof configs extra env mixed large spawn2 rccl
#   fuzz_states fuzz_states_plain fuzz_mixed fuzz_rows fuzz_ingest fuzz_large
#   phase (needs the stamp build: make -C spatial-intention-maps_amd/csrc prof first)
# Environment: SEED0 (fuzz seed base, default 50000).  pytest=a.py,b.py runs those test files instead of tests/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag="$1"; shift
seed0="${SEED0:-50000}"
specs=()
for step in "$@"; do
  name="${step%%=*}"; extra=""
  [ "$name" != "$step" ] && extra="${step#*=}" && extra="${extra//,/ }"
  case "$name" in
    pytest)  c="600|python -u -m pytest ${extra:-tests} -m gpu -x -q --timeout 120 --timeout-method thread"; extra="" ;;
    smoke)   c="120|python -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench)   c="300|python bench.py" ;;
    bench20) c="200|python bench.py --gpus 1 --steps 20 --warmup 5" ;;
    prof)    c="600|bash tools/profile_round.sh $tag" ;;
    configs) c="400|bash tools/bench_configs.sh" ;;
    extra)   c="400|python tools/bench_extra.py" ;;
    env)     c="200|python tools/bench_extra.py --env-step" ;;
    mixed)   c="200|python tools/bench_extra.py --mixed" ;;
    large)   c="200|python tools/bench_extra.py --gridgraph-large" ;;
    spawn2)  c="200|python bench.py --gpus 2 --shared-gpu --steps 100 --warmup 10" ;;
    rccl)    c="200|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --init-dist --steps 50 --no-cpu-baseline" ;;
    fuzz_states)       c="900|SIMAPS_FUZZ_SEED0=$seed0 python tools/fuzz_states.py 256 16 --perturb" ;;
    fuzz_states_plain) c="900|SIMAPS_FUZZ_SEED0=$seed0 python tools/fuzz_states.py 256 16 --perturb --plain" ;;
    fuzz_mixed)        c="900|SIMAPS_FUZZ_SEED0=$seed0 python tools/fuzz_states.py 512 16 --perturb --mixed" ;;
    fuzz_rows)         c="600|python tools/fuzz_rows.py --seed0 $seed0 256 4 16" ;;
    fuzz_ingest)       c="600|SIMAPS_FUZZ_SEED0=$seed0 python tools/fuzz_ingest.py 128 16" ;;
    fuzz_large)        c="600|python tools/fuzz_large.py 96 $seed0" ;;
    phase)   c="120|python tools/phase_profile.py --dump gpurun_out/${tag}_stamps.npy" ;;
    *) echo "unknown step $name" >&2; exit 2 ;;
  esac
  specs+=("${c%%|*}|${tag}_${name}|${c#*|} $extra")
done
bash tools/gpu_session.sh "${specs[@]}"
