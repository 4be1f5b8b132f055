#!/bin/bash
# r03 call 31: stem window-load ring depth (RV_STEM_AHEAD 1 / 7 / 18): stem parity tests,
# bench A/B with the eager conv table (stem launch time)
set -o pipefail
O=${O:-gpurun_out/r03ae}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03ad.json
$T 300 python -u -m pytest tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "stem or first_conv or layerwise or detect" > $O/pytest.log 2>&1 &&
for a in 7 1 18 7 1 18; do
  RV_STEM_AHEAD=$a RV_CONV_TABLE=$O/tab_a$a $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_a$a.json 2> $O/bench_a$a.err || exit 1
  echo "ahead=$a $(python3 -c "
import json;d=json.load(open('$O/bench_a$a.json'));t=json.load(open('$O/tab_a${a}_eager.json'))
st=[round(r['us'],1) for r in t['launches'] if r['conv'].startswith('stem')]
print(d['value'], d.get('device_only',{}).get('value'), d['roofline']['conv_ms_per_step'], 'stem_us', st)")" >> $O/ab.txt
done
rc=$?
tail -2 $O/pytest.log
cat $O/ab.txt
exit $rc
