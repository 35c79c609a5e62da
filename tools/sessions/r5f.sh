# Round-5: large-window sweeps, waves per direction (WPD) x lines prefetched (PF): correctness diff and
# the bench row per build; the product build (WPD 4, PF 16) also through the large-grid tests.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
specs=("400|r5f_pytest_large|python -u -m pytest tests/test_gpu_gridgraph_large.py -x -v --timeout 300 --timeout-method thread")
for v in w4p16 w4p32 w1p32 w1p48 w2p32; do
  specs+=("120|r5f_diff_$v|SIMAPS_LIB=$L/libsimaps_gl$v.so python tools/debug/gl_sssp_diff.py")
  specs+=("200|r5f_extra_$v|SIMAPS_LIB=$L/libsimaps_gl$v.so python tools/bench_extra.py --gridgraph-large")
done
bash tools/gpu_session.sh "${specs[@]}"
