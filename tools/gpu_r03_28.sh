#!/bin/bash
# r03 call 28: single-read preprocess (prep_oneread_kernel) -- parity incl. the repeated
# hand-off test, engine tests, bench A/B against the two-launch form (RV_PREP_ONEREAD=0),
# eager PMC FETCH_SIZE of the preprocess kernels both ways
set -o pipefail
O=${O:-gpurun_out/r03aa}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03y.json
$T 300 python -u -m pytest tests/test_preprocess_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pre.log 2>&1 &&
$T 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_eng.log 2>&1 &&
for g in 1 0 1 0; do
  RV_PREP_ONEREAD=$g $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_o$g.json 2> $O/bench_o$g.err || exit 1
  echo "oneread=$g $(python3 -c "import json;d=json.load(open('$O/bench_o$g.json'));print(d['value'], d.get('device_only',{}).get('value'))")" >> $O/ab.txt
done &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
for g in 1 0; do
  RV_PREP_ONEREAD=$g timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_o$g -o pmc -- python3 tools/pmc_step.py > $O/pmc_o$g.log 2>&1 || exit 1
  find $O/pmc_o$g -name "*counter_collection.csv" -exec mv {} $O/pmc_o$g.csv \;
  rm -rf $O/pmc_o$g
done
rc=$?
tail -2 $O/pytest_pre.log; tail -2 $O/pytest_eng.log
cat $O/ab.txt
for g in 1 0; do python3 - $O/pmc_o$g.csv <<'PY' || true
import csv, sys
rows = {}
for r in csv.DictReader(open(sys.argv[1])):
    rows.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0])[1] += float(r["Counter_Value"])
v = list(rows.values())
for name, val in v[-40:]:
    if any(k in name for k in ("prep_oneread", "clahe_lut", "med3", "letterbox_pad")):
        print(sys.argv[1].split("/")[-1], name.split("(")[0][-40:], round(2 * val / 1024, 1), "MB")
PY
done
exit $rc
