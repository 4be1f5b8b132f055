# NMS / detector / engine GPU tests, NMS timing, then the PMC traffic record
# for this library build (bench.py reads profiles/r05/pmc_traffic.json)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-nmschk}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_detect_gpu.py tests/test_engine_gpu.py tests/test_config5_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 200 python tools/nms_stats.py > $O/nms_stats.txt 2>&1 || exit 1
cat $O/nms_stats.txt | tail -n 2
if [ -n "$PMC" ]; then
  TAG=${O#gpurun_out/}/pmc timeout -k 10 600 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -n 20 $O/pmc.log; exit 1; }
  tail -n 2 $O/pmc.log
fi
