#!/bin/bash
# r03 call 5: fp8 parity with the ordered v8m weights, config-5 fp8 b16, per-layer conv table at
# the bench's B = 128, materialise probe, then the full suite.
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_fp8_gpu.py tests/test_config5_gpu.py > $O/pytest_fp8.log 2>&1 &&
$T 60 python tools/probe_materialise.py > $O/materialise.log 2>&1 &&
RV_CONV_TABLE=$O/conv_table $T 400 python bench.py --steps 20 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err &&
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
exit $rc
