#!/bin/bash
# r03 call 27: frame-grouped preprocess (LUT pass and fused pass alternating per RV_PRE_GROUP
# frames so the fused pass re-reads from the Infinity Cache): parity, bench A/B over group
# sizes (same tuned configs), eager PMC FETCH_SIZE of clahe_lut + med3 per group size
set -o pipefail
O=${O:-gpurun_out/r03z}; mkdir -p $O
export PYTHONUNBUFFERED=1
T="timeout -k 10"
TL=profiles/r03/tune_r03y.json
$T 400 python -u -m pytest tests/test_preprocess_gpu.py tests/test_engine_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 &&
for g in 0 4 2 8 0 4; do
  RV_PRE_GROUP=$g $T 200 python bench.py --steps 20 --tune-load $TL > $O/bench_g$g.json 2> $O/bench_g$g.err || exit 1
  echo "g=$g $(python3 -c "import json;d=json.load(open('$O/bench_g$g.json'));print(d['value'], d.get('device_only',{}).get('value'))")" >> $O/ab.txt
done &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
for g in 0 4; do
  RV_PRE_GROUP=$g timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_g$g -o pmc -- python3 tools/pmc_step.py > $O/pmc_g$g.log 2>&1 || exit 1
  find $O/pmc_g$g -name "*counter_collection.csv" -exec mv {} $O/pmc_g$g.csv \;
  rm -rf $O/pmc_g$g
  python3 tools/pmc_report.py $O/pmc_g$g.csv > $O/pmc_g$g.txt
done
rc=$?
tail -3 $O/pytest.log
cat $O/ab.txt
grep -E "clahe_lut|med3" $O/pmc_g0.txt $O/pmc_g4.txt | head -40
exit $rc
