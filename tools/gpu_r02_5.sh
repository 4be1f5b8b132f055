set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02_gputest5.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL" gpurun_out/r02_gputest5.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --conv-timing none --tune-save gpurun_out/tune5.json > gpurun_out/r02_b5_l1.json 2> gpurun_out/r02_b5_l1.err || exit $?
for L in 2 3; do
  for C in 8 0; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --conv-timing none --tune-load gpurun_out/tune5.json --lanes $L --graph-chunk $C > gpurun_out/r02_b5_l${L}_c$C.json 2> gpurun_out/r02_b5_l${L}_c$C.err || exit $?
  done
done
for f in gpurun_out/r02_b5_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['sort'])"; done
