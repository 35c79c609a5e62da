#!/bin/bash
# Retry a gpurun call only while the pool reports no free slot / box ("transient": nothing ran,
# nothing charged). Any other outcome (ok, fail, refused, timeout) ends the loop.
# usage: gpurun_retry.sh TIMEOUT SCRIPT OUTFILE
t=$1; script=$2; out=$3
case "$t" in ''|*[!0-9]*) echo "usage: $0 TIMEOUT SCRIPT OUTFILE (TIMEOUT in seconds)" >&2; exit 2;; esac
[ -f "$script" ] && [ -n "$out" ] || { echo "usage: $0 TIMEOUT SCRIPT OUTFILE" >&2; exit 2; }
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "bash $script" > "$out" 2>&1
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ]; then echo "attempt $i: $st" >> "$out"; exit 0; fi
  sleep 100
done
echo "gave up after 10 transient attempts" >> "$out"
