#!/bin/bash
# r03 call 9: conv_patch DMA through buffer resources -- parity, then A/B against the previous
# build (librvhip_old.so) with per-layer eager tables.
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$T 600 $P tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_fp8_gpu.py > $O/pytest_conv.log 2>&1 &&
for v in default old default old; do
  RV_LIB_VARIANT=$v RV_CONV_TABLE=$O/tab_$v $T 300 python bench.py --steps 20 --no-cpu-baseline --conv-timing eager > $O/b_$v.json 2> $O/b_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_$v.json'));print('$v', d['value'], d['device_only']['value'], d['roofline']['conv_ms_per_step'], d['roofline']['frac'])" >> $O/ab.txt
done
cat $O/ab.txt
