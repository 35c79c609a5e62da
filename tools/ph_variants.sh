set -e
# Per-phase stamps of the product-equivalent stamp build, then of each ablation variant
# (make prof; make variant NAME=X DEFS=-DSIMAPS_ABL_X).  Run on the GPU box.
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_profile.py > gpurun_out/ph_base.log 2>&1
for v in NOSWEEP NORENDER NORASTER NOGPIX NOGATHER; do
  if [ -f spatial-intention-maps_amd/simaps/libsimaps_$v.so ]; then
    SIMAPS_PROF_LIB=$PWD/spatial-intention-maps_amd/simaps/libsimaps_$v.so timeout -k 10 120 python tools/phase_profile.py > gpurun_out/ph_$v.log 2>&1
  fi
done
