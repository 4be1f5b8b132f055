#!/bin/bash
# r03 call 30: artifacts on the current build -- one single run of the whole GPU suite, smoke,
# the driver's bench line (with CPU baseline and conv tables), a kernel trace of the bench
# command, the PMC traffic passes (profiles/r03/pmc_traffic.json must match this library)
set -o pipefail
O=${O:-gpurun_out/r03ad}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 &&
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
RV_CONV_TABLE=$O/tab $T 500 python bench.py --steps 20 --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err &&
TAG=${TAGP:-r03ad}/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=both $T 400 bash tools/gpu_profile.sh > $O/prof.log 2>&1 &&
TAG=${TAGP:-r03ad}/pmc $T 500 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
