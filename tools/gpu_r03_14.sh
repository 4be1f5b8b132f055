#!/bin/bash
# r03 call 14: fused vs unfused C2f chains, paired vs separate Detect-head branches (per-layer tables)
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing eager"
RV_CONV_TABLE=$O/t_base $T 300 $B > $O/base.json 2> $O/base.err &&
RV_FUSE_C2F=0 RV_CONV_TABLE=$O/t_nofuse $T 300 $B > $O/nofuse.json 2> $O/nofuse.err &&
RV_HEAD_PAIR=0 RV_CONV_TABLE=$O/t_nopair $T 300 $B > $O/nopair.json 2> $O/nopair.err
rc=$?
for f in base nofuse nopair; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'], d['roofline']['conv_ms_per_step'])"; done
exit $rc
