#!/bin/bash
# r03 call 29: single-read pass -- eager time of the pass alone (both forms) and bench
# against the persistent grid size (RV_PREP_WGS)
set -o pipefail
O=${O:-gpurun_out/r03ac}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03y.json
for g in 0 1; do RV_PREP_ONEREAD=$g $T 120 python tools/time_preprocess.py > $O/time_o$g.txt 2>&1 || exit 1; done &&
for w in 256 512 768; do
  RV_PREP_ONEREAD=1 RV_PREP_WGS=$w $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_w$w.json 2> $O/bench_w$w.err || exit 1
  echo "wgs=$w $(python3 -c "import json;d=json.load(open('$O/bench_w$w.json'));print(d['value'], d.get('device_only',{}).get('value'))")" >> $O/ab.txt
done
rc=$?
grep -h "clahe_med_lb" $O/time_o0.txt $O/time_o1.txt
cat $O/ab.txt
exit $rc
