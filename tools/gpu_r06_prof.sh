#!/bin/bash
# Round-6 check + profile on one box: the detector GPU tests, the driver's
# bench (configs saved), a rocprofv3 kernel trace of the same bench
# (timed region + both conv passes, tools/gpu_profile.sh) and the conv
# phase build (tools/conv_phase.py, librvhip_phase.so).  TAG=x bash tools/gpu_r06_prof.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06prof}
mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
if [ -n "${TESTS:-}" ]; then
  $T 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
$T 400 python bench.py --steps 20 --no-cpu-baseline --no-secondary --tune-save $O/tune.json > $O/bench.json \
  2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
TAG=${O#gpurun_out/}/prof TUNE=$O/tune.json STEPS=20 CONV_TIMING=both BENCH_ARGS=--no-secondary \
  $T 400 bash tools/gpu_profile.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -22 $O/prof/timed_summary.txt
if [ -f road-vision-system_amd/rvs_amd/librvhip_phase.so ]; then
  RV_LIB_VARIANT=phase $T 300 python tools/conv_phase.py > $O/phase.txt 2>&1 || { tail $O/phase.txt; exit 1; }
  cat $O/phase.txt
fi
