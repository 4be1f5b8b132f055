#!/bin/bash
# Correctness of the current library on the layer / detector tests, then the
# per-conv eager table (tools/conv_profile.py, B=128 1080p) of two library
# builds alternately: TAG=x VARS="base default base default" bash tools/gpu_conv_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py} -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  tail -n 3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for v in ${VARS:-base default base default}; do
  i=$((i + 1))
  RV_LIB_VARIANT=$v B=${B:-128} timeout -k 10 300 python -u tools/conv_profile.py > $OUT/conv_${i}_$v.log 2>&1 || exit $?
  echo "$v: $(grep "conv sum" $OUT/conv_${i}_$v.log)"
done
