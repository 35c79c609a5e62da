#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tools/micro/fetch_calib.hip, built in-tree as
# tools/micro/fetch_calib): one --pmc pass per counter, each under its own hard limit.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/fetch_calib
mkdir -p "$out"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out" -o fetch -- tools/micro/fetch_calib
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out" -o write -- tools/micro/fetch_calib
echo "calibration in $out"
