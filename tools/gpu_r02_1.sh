set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02_gputest1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r02_gputest1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --tune-save gpurun_out/tune_r02a.json > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err
rc=$?
echo "bench rc=$rc"
cat gpurun_out/r02_bench1.json | head -c 4000
exit $rc
