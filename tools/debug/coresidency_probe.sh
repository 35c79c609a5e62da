cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
V64=spatial-intention-maps_amd/simaps/libsimaps_v64.so
for cfg in lifting_4-small_divider rescue_4-small_empty; do
  for envs in 64 256; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --envs $envs --steps 100 >> gpurun_out/r6f_prod.jsonl || exit $?
    SIMAPS_LIB=$V64 timeout -k 10 120 python bench.py --no-cpu-baseline --config $cfg --envs $envs --steps 100 >> gpurun_out/r6f_v64.jsonl || exit $?
  done
done
