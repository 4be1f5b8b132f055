#!/bin/bash
# Eager per-conv table (tools/conv_profile.py, B = 128) for each library
# variant of VARS (RV_LIB_VARIANT; "default" = librvhip.so), ROUNDS times,
# with the extra environment ENVS; prints the conv sum and the lines of
# layers matching PICK.
#   TAG=x VARS="default nosig" ENVS="RV_HEAD_CHAIN=1" PICK="model.22.cv3.0" bash tools/gpu_conv_variants.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-cv}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARS:-default}; do
    f=$OUT/${v}_$r.log
    env $ENVS RV_LIB_VARIANT=$v B=128 timeout -k 10 300 python -u tools/conv_profile.py > $f 2>&1 || { tail -n 20 $f; exit 1; }
    echo "$v #$r: $(grep 'conv sum' $f)"
    grep -E "${PICK:-model.22.cv3.0}" $f || true
  done
done
