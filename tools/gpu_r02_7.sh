set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02_gputest7.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r02_gputest7.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --tune-save gpurun_out/tune_r02e.json > gpurun_out/r02_bench7.json 2> gpurun_out/r02_bench7.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r02_bench7.err; python3 -c "import json; d=json.load(open('gpurun_out/r02_bench7.json')); print(d['value'], d['ms_per_step'], d['sort'], d['roofline']['conv_ms_per_step'])"
[ $rc -eq 0 ] || exit $rc
TAG=r02_prof7 TUNE=gpurun_out/tune_r02e.json bash tools/gpu_profile.sh
