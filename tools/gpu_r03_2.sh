#!/bin/bash
# r03 call 2: the native launch list -- engine parity tests, bench A/B at --steps 20, full suite.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_engine.log 2>&1 &&
for m in "native --sync flow" "native --sync stage" "eager --sync flow" "graph"; do
  tag=$(echo $m | tr -d ' -')
  $T 300 python bench.py --steps 20 --exec $m --no-cpu-baseline --conv-timing none > $O/bench_$tag.json 2> $O/bench_$tag.err || exit 1
done &&
$T 300 python bench.py --steps 60 --exec native --sync flow --no-cpu-baseline --conv-timing none > $O/bench_native60.json 2> $O/bench_native60.err &&
$T 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
exit $rc
