#!/bin/bash
# r03 call 1: eager vs graph pipelined bench at the driver's --steps 20, then the GPU suite
# with per-test names and the native crash handler.
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 20 --exec eager --no-cpu-baseline --conv-timing none > $O/bench_eager.json 2> $O/bench_eager.err &&
timeout -k 10 300 python bench.py --steps 20 --exec graph --no-cpu-baseline --conv-timing none > $O/bench_graph.json 2> $O/bench_graph.err &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
exit $rc
