#!/bin/bash
# r03 call 16: fast epilogue + C2f fusion level 1 (C = 16 only): parity, then the bench line
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 800 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_fp8_gpu.py tests/test_engine_gpu.py tests/test_config5_gpu.py > $O/pytest.log 2>&1 &&
RV_CONV_TABLE=$O/tab $T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing eager > $O/bench.json 2> $O/bench.err
rc=$?
tail -2 $O/pytest.log
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['device_only']['value'], d['roofline']['conv_ms_per_step'])"
exit $rc
