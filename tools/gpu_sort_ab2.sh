#!/bin/bash
# SORT forms A/B on one box: the GPU SORT / engine tests, the isolated
# rv_sort_update timing (tools/time_sort.py) of the three-launch form and
# the fused one-launch form alternately, then the driver's bench A/B
# (tools/gpu_ab2.sh).   TAG=x bash tools/gpu_sort_ab2.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sortab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_sort_gpu.py tests/test_track_ops_gpu.py tests/test_engine_gpu.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for f in 0 1 0 1; do
  echo "RV_SORT_FUSED=$f: $(RV_SORT_FUSED=$f timeout -k 10 120 python tools/time_sort.py 32 40 2>&1 | tail -n 1)"
done
TAG=$TAG/bench ROUNDS=${ROUNDS:-3} CONFIGS=$'sort3;RV_SORT_FUSED=0\nsortf;RV_SORT_FUSED=1' bash tools/gpu_ab2.sh
