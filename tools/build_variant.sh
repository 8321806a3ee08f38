#!/bin/bash
# Build an alternative libgbv (same sources, extra compiler defines) for A/B runs:
#   bash tools/build_variant.sh <name> -DGBV_WAVES_PER_EU=1 ...  -> lodestar_amd/variants/libgbv_<name>.so
# select it with LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_<name>.so
set -e
NAME=$1; shift
OUT=lodestar_amd/variants
mkdir -p $OUT/obj_$NAME
for f in lodestar_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $f -o $OUT/obj_$NAME/$b.o &
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgbv_$NAME.so $OUT/obj_$NAME/*.o
rm -rf $OUT/obj_$NAME
echo built $OUT/libgbv_$NAME.so
