set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sort_gpu.py tests/test_track_ops_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r02_sorttest8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r02_sorttest8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/time_sort.py 32 40 || exit $?
timeout -k 10 120 python -u tools/time_sort.py 32 80 || exit $?
