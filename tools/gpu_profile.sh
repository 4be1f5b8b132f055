# rocprofv3 kernel trace of bench.py's timed region (tools/trace_window.py
# keeps the dispatches between the rv_trace_marker kernels), with the conv
# configs saved by a preceding `bench.py --tune-save $TUNE` so no autotuner
# launch is in the trace.  usage: TAG=r02 TUNE=gpurun_out/tune.json bash tools/gpu_profile.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-prof}
STEPS=${STEPS:-60}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/raw" -o trace -- \
  python3 bench.py --tune-load "$TUNE" --warmup 1 --steps "$STEPS" --no-cpu-baseline \
  --conv-timing ${CONV_TIMING:-none} ${BENCH_ARGS:-} > "$OUT/bench_profiled.json" \
  2> "$OUT/bench_profiled.err" || exit $?
KT=$(find "$OUT/raw" -name "*kernel_trace.csv" | head -1)
ST=$(find "$OUT/raw" -name "*kernel_stats.csv" | head -1)
cp "$ST" "$OUT/rocprof_kernel_stats_whole_run.csv"
python3 tools/trace_window.py "$KT" "$STEPS" "$OUT/timed" || exit $?
python3 tools/stream_busy.py "$KT" "$STEPS" > "$OUT/timed_streams.txt" || exit $?
python3 tools/timeline.py "$KT" 1,2 250 > "$OUT/timed_timeline.txt" || exit $?
if grep -q "device-only" "$OUT/bench_profiled.json" 2>/dev/null; then  # the device-only rerun
  python3 tools/trace_window.py "$KT" "$STEPS" "$OUT/devonly" 7,8 > /dev/null || exit $?
  python3 tools/stream_busy.py "$KT" "$STEPS" 7,8 > "$OUT/devonly_streams.txt" || exit $?
  python3 tools/timeline.py "$KT" 7,8 250 > "$OUT/devonly_timeline.txt" || exit $?
fi
if [ "${CONV_TIMING:-none}" = both ]; then  # the conv profiling passes' windows
  python3 tools/trace_window.py "$KT" "$STEPS" "$OUT/convpass_pipeline" 3,4 > /dev/null || exit $?
  python3 tools/trace_window.py "$KT" "$STEPS" "$OUT/convpass_eager" 5,6 > /dev/null || exit $?
fi
gzip -c "$KT" > "$OUT/kernel_trace.csv.gz"
rm -rf "$OUT/raw"
