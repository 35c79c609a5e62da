#!/bin/bash
# Build libsimaps.so and the two diagnostic builds in parallel, then check that every library carries
# this tree's source hash (simaps._lib refuses any that does not).
cd "$(dirname "$0")/.."
C=spatial-intention-maps_amd/csrc
make -s -C $C & make -s -j2 -C $C diag & wait
want=$(python3 spatial-intention-maps_amd/simaps/_srchash.py)
rc=0
for f in spatial-intention-maps_amd/simaps/libsimaps.so spatial-intention-maps_amd/simaps/libsimaps_diag*.so; do
  got=$(python3 -c "import ctypes; L=ctypes.CDLL('$f'); L.simaps_source_hash.restype=ctypes.c_char_p; print(L.simaps_source_hash().decode())")
  if [ "$got" != "$want" ]; then echo "STALE: $f"; rc=1; fi
done
[ $rc -eq 0 ] && echo "all libraries built from ${want:0:16}"
exit $rc
