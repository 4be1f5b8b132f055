#!/bin/bash
# Round artifacts on the current build, one GPU box: the whole -m gpu suite
# once, smoke(), the driver's bench command (conv tables, tuned configs saved),
# a rocprofv3 kernel trace of the same bench (timed region, both conv passes,
# the device-only rerun: tools/gpu_profile.sh) and the PMC passes on the same
# tuned configs (tools/gpu_pmc.sh -> pmc_traffic.json for this library).
# Every GPU step has its own time limit; the first failure ends the script.
#   O=gpurun_out/r04x bash tools/gpu_artifacts.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r04art}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
if [ "${TESTS:-1}" = 1 ]; then
  $T 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
  $T 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
fi
RV_CONV_TABLE=$O/tab $T 500 python bench.py --steps 20 --tune-save "$O/tune.json" \
  > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cut -c1-300 "$O/bench.json"
TAG=${O#gpurun_out/}/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=both BENCH_ARGS=--no-secondary \
  $T 400 bash tools/gpu_profile.sh > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
head -3 "$O/prof/timed_summary.txt"
TAG=${O#gpurun_out/}/pmc TUNE=$O/tune.json $T 600 bash tools/gpu_pmc.sh > "$O/pmc.log" 2>&1 ||
  { tail -20 "$O/pmc.log"; exit 1; }
tail -3 "$O/pmc.log"
