#!/bin/bash
# r03 call 11: i8-MFMA conv0 + restructured stem -- layer / detect / fp8 / engine parity, smoke,
# then the bench with the per-layer conv tables.
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_fp8_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1 &&
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
RV_CONV_TABLE=$O/tab $T 400 python bench.py --steps 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest.log
exit $rc
