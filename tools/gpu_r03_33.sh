#!/bin/bash
# r03 call 33: pipeline unit size at the driver's --steps 20 (RV_PAIR 4 / 2 / 5), alternating
set -o pipefail
O=${O:-gpurun_out/r03ag}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03ad.json
for p in 4 2 5 4 2 5; do
  RV_PAIR=$p $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_p$p.json 2> $O/bench_p$p.err || exit 1
  echo "pair=$p $(python3 -c "
import json;d=json.load(open('$O/bench_p$p.json'))
print(d['value'], d.get('device_only',{}).get('value'), d.get('steady_state_frames_per_s'), d['config'].get('pair', d['config'].get('steps_per_unit')))")" >> $O/ab.txt
done
rc=$?
cat $O/ab.txt
exit $rc
