set -e
for v in NOSWEEP NORASTER NOGPIX NOGATHER; do
  SIMAPS_PROF_LIB=$PWD/spatial-intention-maps_amd/simaps/libsimaps_$v.so timeout -k 10 120 python tools/phase_profile.py > gpurun_out/ph_$v.log 2>&1
done
