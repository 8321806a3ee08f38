#!/bin/bash
# Build an alternative libgbv (same sources, extra compiler defines) for A/B runs:
#   bash tools/build_variant.sh <name> -DGBV_WAVES_PER_EU=1 ...  -> lodestar_amd/variants/libgbv_<name>.so
# select it with LODESTAR_AMD_LIB=lodestar_amd/variants/libgbv_<name>.so
set -e
NAME=$1; shift
OUT=lodestar_amd/variants
mkdir -p $OUT/obj_$NAME
export FLAGS="$*" OBJ=$OUT/obj_$NAME
ls lodestar_amd/csrc/*.hip | xargs -P 6 -I{} sh -c 'hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS -c {} -o $OBJ/$(basename {} .hip).o 2>/dev/null || { echo "FAILED {}"; exit 1; }'
hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgbv_$NAME.so $OUT/obj_$NAME/*.o
rm -rf $OUT/obj_$NAME
echo built $OUT/libgbv_$NAME.so
