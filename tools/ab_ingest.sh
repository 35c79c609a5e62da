# Ingest kernel A/B on the GPU box: libsimaps_base.so (a build of another revision, made by hand) against
# the product libsimaps.so, alternating twice (tools/bench_extra.py --ingest-only: kernels alone).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for lib in libsimaps_base.so libsimaps.so; do
  SIMAPS_LIB=$PWD/spatial-intention-maps_amd/simaps/$lib timeout -k 10 120 python tools/bench_extra.py --ingest-only > gpurun_out/ing_$lib.$rep.log 2>&1 || exit 1
  grep '^{' gpurun_out/ing_$lib.$rep.log | python -c "import json,sys; d=json.load(sys.stdin); print('$lib', round(d['gpu_ms_per_launch']*1e3,1), 'us', round(d['roofline']['frac'],3))"
done
done
