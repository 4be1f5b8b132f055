#!/bin/bash
# Per-layer kernel time of the YOLOv8 forward under each forced patch tile
# (RV_CONV_FORCE=MR,NR) with and without persistence; one rocprofv3 kernel
# trace per config under gpurun_out/sweep/.  Summarize with tools/sweep_table.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep
for p in 1 0; do
  for f in auto 1,1 1,2 1,4 2,1 2,2 2,4 4,1 4,2 4,4 8,1 8,2; do
    tag="${f/,/x}_p$p"
    if [ "$f" = auto ]; then unset RV_CONV_FORCE; else export RV_CONV_FORCE=$f; fi
    RV_CONV_PERSIST=$p N=3 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/sweep/$tag -o t \
      -- python3 tools/trace_forward.py > gpurun_out/sweep/$tag.log 2>&1
    python3 tools/sweep_table.py --dump gpurun_out/sweep/$tag > gpurun_out/sweep/$tag.txt
    rm -rf gpurun_out/sweep/$tag
    echo "$tag $(grep forward gpurun_out/sweep/$tag.log)"
  done
done
