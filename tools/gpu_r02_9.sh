set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py -m gpu -v --timeout 200 --timeout-method thread -x > gpurun_out/r02_c2ftest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/r02_c2ftest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --tune-save gpurun_out/tune9.json > gpurun_out/r02_b9.json 2> gpurun_out/r02_b9.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r02_b9.json')); print(d['value'], d['ms_per_step'], d['roofline']['conv_ms_per_step'], d['roofline']['launches_per_step'])"
TAG=r02_prof9 TUNE=gpurun_out/tune9.json bash tools/gpu_profile.sh
