#!/bin/bash
# Round-end style pass on one GPU box: the whole -m gpu suite, smoke(), the
# default bench line (tuned configs saved), the rocprofv3 trace of the same
# bench (timed window + both conv passes), and the PMC passes.  Each GPU step
# has its own time limit; the first failure ends the script.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py --tune-save "$OUT/tune.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
cut -c1-200 "$OUT/bench.json"
TAG=${TAG:-round}/prof TUNE="$OUT/tune.json" CONV_TIMING=both timeout -k 10 400 bash tools/gpu_profile.sh \
  > "$OUT/prof.log" 2>&1
head -3 "$OUT/prof/timed_summary.txt"
TAG=${TAG:-round}/pmc timeout -k 10 700 bash tools/gpu_pmc.sh > "$OUT/pmc.log" 2>&1
tail -3 "$OUT/pmc.log"
