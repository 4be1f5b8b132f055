#!/bin/bash
# r03 call 17: register-weight 3x3 kernel -- autotune bit-identity + layer parity, then the
# bench line with per-layer tables and the autotuner's per-launch choices
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py > $O/pytest.log 2>&1 &&
RV_CONV_DEBUG=1 RV_CONV_TABLE=$O/tab $T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing eager --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err
rc=$?
tail -2 $O/pytest.log
grep autotune $O/bench.err | head -60 > $O/autotune.txt
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['device_only']['value'], d['roofline']['conv_ms_per_step'])"
exit $rc
