#!/bin/bash
# r03 call 34: untimed warm runs of the recorded schedule before the timed region (1 vs 3)
set -o pipefail
O=${O:-gpurun_out/r03ah}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03ad.json
i=0
for w in 1 3 1 3 1 3 1 3; do
  i=$((i + 1))
  RV_WARM_RUNS=$w $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "warm_runs=$w $(python3 -c "
import json;d=json.load(open('$O/bench_$i.json'));print(d['value'], d.get('device_only',{}).get('value'))")" >> $O/ab.txt
done
rc=$?
cat $O/ab.txt
exit $rc
