# Round-4 overlapped early-exit path kernel (OVL, simaps_path_mode 3; the automatic mode's choice for
# launches resident at once): the path tests first, then all GPU tests, smoke, the path bench in all
# three modes (+ stamps), the env step under a kernel trace, a fresh-seed fuzz in mode 3, the headline.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "240|r4s_pytest_paths|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'path or spfa or overlap or gridgraph'" \
  "420|r4s_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r4s_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|r4s_pathbench|python tools/path_bench.py" \
  "300|r4s_pathbench_stamps|python tools/path_bench.py --stamps" \
  "300|r4s_extra|python tools/bench_extra.py" \
  "200|r4s_envstep_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s_prof -o envstep -- python tools/bench_extra.py --env-step" \
  "300|r4s_rows_fuzz|python tools/fuzz_rows.py --path-mode 3 128 4 16" \
  "300|r4s_bench|python bench.py"
