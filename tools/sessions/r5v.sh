# Round-5: the ingest key map's and the receptacle cache's stream ordering without per-call events --
# the drop-in tests (ingest, graph capture, cross-stream cache), then the 8(f) rows.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "400|r5v_pytest_dropin|python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_mixed.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|r5v_extra|python tools/bench_extra.py" \
  "200|r5v_env|python tools/bench_extra.py --env-step"
