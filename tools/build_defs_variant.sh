#!/bin/bash
# Build librvhip.so of the WORKING TREE with extra preprocessor defines as an
# A/B variant: NAME=burst DEFS="-DRV_DMA_BURST" bash tools/build_defs_variant.sh
#   -> road-vision-system_amd/rvs_amd/librvhip_burst.so (RV_LIB_VARIANT=burst)
set -eo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=${NAME:?}
TMP=$(mktemp -d /tmp/rvdef.XXXXXX)
mkdir -p "$TMP/road-vision-system_amd/rvs_amd" "$TMP/include"
cp -r "$REPO/road-vision-system_amd/csrc" "$TMP/road-vision-system_amd/"
rm -rf "$TMP/road-vision-system_amd/csrc/build"
cp "$REPO/include/"*.h "$TMP/include/"
make -C "$TMP/road-vision-system_amd/csrc" -j8 HIPCC="/opt/rocm/bin/hipcc $DEFS" ../rvs_amd/librvhip.so \
  > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
cp "$TMP/road-vision-system_amd/rvs_amd/librvhip.so" "$REPO/road-vision-system_amd/rvs_amd/librvhip_$NAME.so"
rm -rf "$TMP"
echo "built librvhip_$NAME.so with $DEFS"
