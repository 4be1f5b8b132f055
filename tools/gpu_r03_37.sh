#!/bin/bash
# r03 call 37: final-HEAD check -- whole GPU suite once, smoke, the driver's bench command
set -o pipefail
O=${O:-gpurun_out/r03ak}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 &&
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$T 500 python bench.py --steps 20 > $O/bench.json 2> $O/bench.err
rc=$?
tail -2 $O/pytest_gpu.log
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d.get('warm_runs'))" || true
exit $rc
