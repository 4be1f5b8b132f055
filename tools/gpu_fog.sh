#!/bin/bash
# Config-5 bench with the full fog chain vs the core pass, and a kernel trace
# of the full chain (fog kernels' per-launch durations).
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-fog}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/bench_config5.py --fog full --cpu-frames ${CPU_FRAMES:-0} > "$OUT/bench_config5_full.json" 2> "$OUT/full.err"
cat "$OUT/bench_config5_full.json"
timeout -k 10 300 python -u tools/bench_config5.py --fog core --cpu-frames 0 > "$OUT/bench_config5_core.json" 2> "$OUT/core.err"
cat "$OUT/bench_config5_core.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o fog -- \
  python3 tools/bench_config5.py --fog full --cpu-frames 0 --steps 5 --autotune 0 > "$OUT/prof.json" 2> "$OUT/prof.err"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/fog_kernel_stats.csv" \;
rm -rf "$OUT/prof"
