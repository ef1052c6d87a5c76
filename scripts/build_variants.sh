#!/bin/bash
# build_variants.sh NAME "-DFLAGS" [NAME "-DFLAGS" ...]: _variants/NAME.so each with the Makefile's
# register budgets plus the extra flags (scripts/build_variant.sh)
cd "$(dirname "$0")/.."
D="-DRS_TRAV_INLINE=1 -DRS_INITIAL_WAVES=5 -DRS_SPATIAL_WAVES=4 -DRS_SPATIAL_WAVES_SMALL=5 -DRS_INITIAL_WAVES_LANE=7 -DRS_SPATIAL_WAVES_LANE=6 -DRS_TEMPORAL_WAVES_LANE=6"
while [ $# -ge 2 ]; do
  bash scripts/build_variant.sh "$1" "$D $2" > /tmp/bv_$1.log 2>&1 || echo "build $1 failed"
  shift 2
done
ls restir-embree_amd/_variants/*.so
