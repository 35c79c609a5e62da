#!/bin/bash
# Build the phase-stamp library of a git revision as spatial-intention-maps_amd/simaps/libsimaps_<NAME>.so
# (A/B timing within one GPU call: tools/diag_variants.sh NAME1 NAME2 NAME1 NAME2).
#   tools/ab_build.sh <rev> <name> [extra -D flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
git -C "$ROOT" show "$rev:spatial-intention-maps_amd/csrc/simaps.hip" > "$tmp/simaps.hip"
git -C "$ROOT" show "$rev:spatial-intention-maps_amd/csrc/geom.h" > "$tmp/geom.h"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fPIC -shared -I"$ROOT/include" -I"$tmp" \
    -DSIMAPS_PHASE_STAMPS "$@" "$tmp/simaps.hip" -o "$ROOT/spatial-intention-maps_amd/simaps/libsimaps_$name.so"
rm -rf "$tmp"
