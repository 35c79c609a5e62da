# Round-5: (1) debug of gl_sssp_kernel (large-window images differ from the oracle in r5b): the product
# build and three debug builds (12 forced rounds / one sweep wave at a time / both);
# (2) timing experiment for the SPFA pop: libsimaps_xread.so issues the next
# pop's LDS reads before this pop's writes with NO forwarding (results invalid; only ns per pop is
# read), against the stamp build of the product pop.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=spatial-intention-maps_amd/simaps
bash tools/gpu_session.sh \
  "120|r5c_gl_diff|python tools/debug/gl_sssp_diff.py" \
  "120|r5c_gl_force|SIMAPS_LIB=$L/libsimaps_glforce.so python tools/debug/gl_sssp_diff.py" \
  "120|r5c_gl_serial|SIMAPS_LIB=$L/libsimaps_glserial.so python tools/debug/gl_sssp_diff.py" \
  "120|r5c_gl_both|SIMAPS_LIB=$L/libsimaps_glboth.so python tools/debug/gl_sssp_diff.py" \
  "150|r5c_prof_1|python tools/path_bench.py --stamps --latency" \
  "150|r5c_xread_1|SIMAPS_PROF_LIB=$L/libsimaps_xread.so python tools/path_bench.py --stamps --latency" \
  "150|r5c_prof_2|python tools/path_bench.py --stamps --latency" \
  "150|r5c_xread_2|SIMAPS_PROF_LIB=$L/libsimaps_xread.so python tools/path_bench.py --stamps --latency"
