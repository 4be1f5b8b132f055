#!/bin/bash
# r03 call 3: new bench (consumer thread, device-only rerun, steady state, multi-core CPU
# baseline) at the driver's --steps 20, then the full GPU suite.
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_engine.log 2>&1 &&
$T 600 python bench.py --steps 20 > $O/bench20.json 2> $O/bench20.err &&
$T 300 python bench.py --steps 20 --pair 2 --no-cpu-baseline --conv-timing none > $O/bench20_p2.json 2> $O/bench20_p2.err &&
$T 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
exit $rc
