set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g64
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/g64/pytest.log 2>&1
tail -3 gpurun_out/g64/pytest.log
SKIP_TRACE=1 VAR=RV_LIB_VARIANT VALS="old default old default" TAG=g64 bash tools/ab_env.sh
