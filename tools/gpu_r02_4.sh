set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02_gputest4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r02_gputest4.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --tune-save gpurun_out/tune_r02d.json > gpurun_out/r02_bench4.json 2> gpurun_out/r02_bench4.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r02_bench4.err; cat gpurun_out/r02_bench4.json
