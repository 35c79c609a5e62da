#!/bin/bash
# Run GPU steps in order on the gpurun box.  Each step has its own time limit.  An ordinary
# failure (exit 1/2, e.g. a failing test) moves on to the next step; a timeout, abort, segfault
# or kill (124, 134, 137, 139, >128) ends the session so nothing else touches the GPU.
# usage: tools/gpu_session.sh "<secs>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "=== stopping: fatal rc=$rc" | tee -a gpurun_out/session.log; exit $rc; fi
done
exit $status
