#!/bin/bash
# r03 call 32: MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form=1 on conv.hip /
# c2f.hip, librvhip_vf.so) vs the default build: layer / detect parity on the vf build,
# bench A/B alternating builds with the eager conv table
set -o pipefail
O=${O:-gpurun_out/r03af}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03ad.json
RV_LIB_VARIANT=vf $T 400 python -u -m pytest tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py tests/test_fp8_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_vf.log 2>&1 &&
for v in default vf default vf default vf; do
  RV_LIB_VARIANT=$v RV_CONV_TABLE=$O/tab_$v $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  echo "lib=$v $(python3 -c "
import json;d=json.load(open('$O/bench_$v.json'));t=json.load(open('$O/tab_${v}_eager.json'))
st=[round(r['us'],1) for r in t['launches'] if r['conv'].startswith('stem')]
print(d['value'], d.get('device_only',{}).get('value'), d['roofline']['conv_ms_per_step'], 'stem_us', st)")" >> $O/ab.txt
done
rc=$?
tail -2 $O/pytest_vf.log
cat $O/ab.txt
exit $rc
