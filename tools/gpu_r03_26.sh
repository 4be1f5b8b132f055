#!/bin/bash
# r03 call 26: the three-stage DMA ring (ConvCfg kind 2) -- every candidate bit-identical
# to the default (autotune verify), the layer / detect tests, then the bench with the
# autotuner's candidate dump and the per-layer conv table
set -o pipefail
O=${O:-gpurun_out/r03x}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
RV_CONV_DEBUG=2 RV_CONV_TABLE=$O/tab $T 400 python bench.py --steps 20 --tune-save $O/tune.json > $O/bench.json 2> $O/bench.err &&
$T 300 python bench.py --steps 20 --tune-load $O/tune.json > $O/bench2.json 2> $O/bench2.err
rc=$?
tail -3 $O/pytest.log
cat $O/bench.json $O/bench2.json 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['value'], d.get('device_only',{}).get('value') if isinstance(d.get('device_only'),dict) else '', d['roofline']['frac'])" || true
exit $rc
