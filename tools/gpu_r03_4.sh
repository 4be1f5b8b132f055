#!/bin/bash
# r03 call 4: consumer in the timed region with the faster to_detections; event wait poll vs
# sync; --steps 20 and 60.
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --no-cpu-baseline --conv-timing none"
$T 300 $B --steps 20 > $O/b20_poll.json 2> $O/b20_poll.err &&
RV_SCHED_WAIT=sync $T 300 $B --steps 20 > $O/b20_sync.json 2> $O/b20_sync.err &&
$T 300 $B --steps 20 --exec eager > $O/b20_eager.json 2> $O/b20_eager.err &&
$T 300 $B --steps 60 > $O/b60_poll.json 2> $O/b60_poll.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
$T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; &&
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \; &&
rm -rf $O/prof && gzip -f $O/kernel_trace.csv &&
$T 240 python3 -u tools/repro_graph_crash.py 4 400 multi > $O/repro_multi.log 2>&1
