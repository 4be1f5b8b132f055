#!/bin/bash
# A/B of library builds on one box (tools/build_variant.sh makes the
# variants): optional parity tests on the default build, then interleaved
# bench runs per variant (REPS rounds) with the per-conv eager tables, then
# one FETCH_SIZE / WRITE_SIZE PMC pass per variant (conv-family traffic).
#   TAG=r04a VARIANTS="base default" TESTS="tests/test_yolo_layers_gpu.py" bash tools/gpu_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
T="timeout -k 10"
if [ -n "${TESTS:-}" ]; then
  $T ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
for rep in $(seq 1 "${REPS:-2}"); do
  for v in ${VARIANTS:-base default}; do
    RV_LIB_VARIANT=$v RV_CONV_TABLE=$O/tab_${v}_$rep $T 300 python -u bench.py --steps ${STEPS:-20} \
      --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err" ||
      { tail -20 "$O/bench_${v}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));r=d['roofline'];print('$v', d['value'], d['ms_per_step'], d.get('device_only',{}).get('value'), r['conv_ms_per_step'], r['frac'], r.get('in_pipeline',{}).get('conv_ms_per_step'))"
  done
done
[ "${PMC:-1}" = 1 ] || exit 0
for v in ${PMC_VARIANTS:-${VARIANTS:-base default}}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RV_LIB_VARIANT=$v timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${v}_$c" \
      -o pmc -- python3 tools/pmc_step.py > "$O/pmc_${v}_$c.log" 2>&1 || { tail "$O/pmc_${v}_$c.log"; exit 1; }
    find "$O/pmc_${v}_$c" -name "*counter_collection.csv" -exec mv {} "$O/pmc_${v}_$c.csv" \;
    rm -rf "$O/pmc_${v}_$c"
  done
  python3 tools/pmc_family.py "$O/pmc_family_$v.json" "$O/pmc_${v}_FETCH_SIZE.csv" \
    "$O/pmc_${v}_WRITE_SIZE.csv" > "$O/pmc_family_$v.txt"
  rm -f "$O"/pmc_${v}_*.csv
  echo "== $v"; grep -E "conv_patch|conv1x1|c2f|stem" "$O/pmc_family_$v.txt" | sed "s/mfma_util.*read_bytes/read_bytes/; s/SQ_INSTS.*//"
done
