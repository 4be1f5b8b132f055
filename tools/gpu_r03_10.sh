#!/bin/bash
# r03 call 10 (after the container restore): one single run of the whole GPU suite, smoke, the
# driver's bench line, a kernel trace of the bench command, and the PMC traffic passes.
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 &&
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$T 400 python bench.py --steps 20 --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err &&
TAG=r03j/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=both $T 400 bash tools/gpu_profile.sh > $O/prof.log 2>&1 &&
TAG=r03j/pmc $T 500 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
