#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, a rocprofv3 kernel
# summary of the same bench command, and the per-conv HIP-event table.
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
  python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
timeout -k 10 200 python3 tools/conv_profile.py > "$OUT/conv_profile.txt" 2>&1
head -50 "$OUT/conv_profile.txt"
