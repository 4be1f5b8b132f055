#!/bin/bash
# r03 call 35: stage-stream priorities (RV_HIPRI_STREAMS: Y1 = sy, Y2 = sm, T = st at high
# priority, the preprocess stream sp at default) against the default, alternating
set -o pipefail
O=${O:-gpurun_out/r03ai}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03ad.json
i=0
for h in none sy,sm,st sm,st none sy,sm,st sm,st; do
  i=$((i + 1))
  if [ "$h" = none ]; then unset RV_HIPRI_STREAMS; else export RV_HIPRI_STREAMS=$h; fi
  $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "hipri=$h $(python3 -c "
import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d.get('device_only',{}).get('value'), d.get('steady_state_frames_per_s'))")" >> $O/ab.txt
done
rc=$?
cat $O/ab.txt
exit $rc
