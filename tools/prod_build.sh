#!/bin/bash
# Product build of a git revision (or the working tree with rev "WT") as
# spatial-intention-maps_amd/simaps/libsimaps_prod_<NAME>.so, for tools/ab_bench.sh.
#   tools/prod_build.sh <rev|WT> <name> [extra -D flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
if [ "$rev" = WT ]; then cp "$ROOT/spatial-intention-maps_amd/csrc/simaps.hip" "$ROOT/spatial-intention-maps_amd/csrc/geom.h" "$tmp/"; else
git -C "$ROOT" show "$rev:spatial-intention-maps_amd/csrc/simaps.hip" > "$tmp/simaps.hip"
git -C "$ROOT" show "$rev:spatial-intention-maps_amd/csrc/geom.h" > "$tmp/geom.h"
git -C "$ROOT" show "$rev:include/simaps.h" > "$tmp/simaps.h"; fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fPIC -shared -I"$tmp" -I"$ROOT/include" \
    "$@" "$tmp/simaps.hip" -o "$ROOT/spatial-intention-maps_amd/simaps/libsimaps_prod_$name.so"
rm -rf "$tmp"
