#!/bin/bash
# r03 call 15: buffer-store conv epilogue (parity + per-layer A/B against RV_EPI_SLOW), fused vs
# unfused C2f chains, paired vs separate Detect-head branches
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py > $O/pytest.log 2>&1 &&
B="python bench.py --steps 20 --no-cpu-baseline --conv-timing eager"
RV_CONV_TABLE=$O/t_base $T 300 $B > $O/base.json 2> $O/base.err &&
RV_EPI_SLOW=1 RV_CONV_TABLE=$O/t_slow $T 300 $B > $O/slow.json 2> $O/slow.err &&
RV_FUSE_C2F=0 RV_CONV_TABLE=$O/t_nofuse $T 300 $B > $O/nofuse.json 2> $O/nofuse.err &&
RV_HEAD_PAIR=0 RV_CONV_TABLE=$O/t_nopair $T 300 $B > $O/nopair.json 2> $O/nopair.err
rc=$?
tail -2 $O/pytest.log
for f in base slow nofuse nopair; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['device_only']['value'], d['roofline']['conv_ms_per_step'])"; done
exit $rc
