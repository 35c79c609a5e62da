# Round-4 path pop v6 (v5 + the early-exit target checks inside the asm loop) as the product:
# all GPU tests, smoke, per-pop stamps, path bench, A/B against the round-3 pop and v5, fresh-seed
# path fuzz; then the headline bench and the 8(f) rows (env step under a kernel trace) on this tree.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "420|r4m_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120|r4m_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|r4m_pathbench_stamps|python tools/path_bench.py --stamps" \
  "200|r4m_pathbench|python tools/path_bench.py" \
  "200|r4m_path_ab|for r in 1 2; do for l in prod_r3pop prod_asmv5; do SIMAPS_LIB=$P/libsimaps_\$l.so python tools/path_ab.py; done; python tools/path_ab.py; done" \
  "300|r4m_rows_fuzz|python tools/fuzz_rows.py 128 4 16" \
  "300|r4m_bench|python bench.py" \
  "400|r4m_extra|python tools/bench_extra.py" \
  "200|r4m_envstep_prof|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m_prof -o envstep -- python tools/bench_extra.py --env-step"
