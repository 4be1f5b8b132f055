set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02_gputest3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r02_gputest3.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --tune-save gpurun_out/tune_r02c.json > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r02_bench3.err; cat gpurun_out/r02_bench3.json
[ $rc -eq 0 ] || exit $rc
TAG=r02_prof3 TUNE=gpurun_out/tune_r02c.json bash tools/gpu_profile.sh
