#!/bin/bash
# Build librvhip.so of a git revision as an A/B variant next to the current
# build: NAME=base REV=HEAD bash tools/build_variant.sh
#   -> road-vision-system_amd/rvs_amd/librvhip_base.so (RV_LIB_VARIANT=base)
set -eo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=${NAME:-base}
REV=${REV:-HEAD}
TMP=$(mktemp -d /tmp/rvvar.XXXXXX)
git -C "$REPO" archive "$REV" road-vision-system_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$TMP/road-vision-system_amd/rvs_amd"
make -C "$TMP/road-vision-system_amd/csrc" -j8 ../rvs_amd/librvhip.so > "$TMP/build.log" 2>&1 ||
  { tail -20 "$TMP/build.log"; exit 1; }
cp "$TMP/road-vision-system_amd/rvs_amd/librvhip.so" "$REPO/road-vision-system_amd/rvs_amd/librvhip_$NAME.so"
rm -rf "$TMP"
echo "built librvhip_$NAME.so from $REV"
