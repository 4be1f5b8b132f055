set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest_engine.log 2>&1
rc=$?
tail -5 gpurun_out/r05a/pytest_engine.log
[ $rc -eq 0 ] || exit $rc
B=128 timeout -k 10 300 python -u tools/conv_profile.py > gpurun_out/r05a/conv_profile_b128.log 2>&1
tail -45 gpurun_out/r05a/conv_profile_b128.log
