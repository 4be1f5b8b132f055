#!/bin/bash
# r03 call 13: virtual-concat neck (no materialised upsamples) + unequal pipeline units --
# layer / detect / engine parity, then a unit-size A/B at the driver's --steps 20.
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 700 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 &&
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing none"
RV_CONV_TABLE=$O/tab $T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing eager --tune-save $O/tune.json > $O/even.json 2> $O/even.err &&
for u in ramp 1,3,4,4,4,3,1 2,4,4,4,4,2 1,2,4,4,4,4,1 1,1,2,4,4,4,2,1,1; do
  $T 300 $B --tune-load $O/tune.json --units $u > $O/u_$u.json 2> $O/u_$u.err || exit 1
done
rc=$?
tail -3 $O/pytest.log
for f in $O/even.json $O/u_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['device_only']['value'], d.get('steady_state_frames_per_s'))"; done
exit $rc
