set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x; mkdir -p $O
for v in default a256; do
  RV_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_sort_gpu.py tests/test_track_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -n 20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/pytest_$v.log)"
done
for r in 1 2; do for v in base default a256; do
  echo "$v: $(RV_LIB_VARIANT=$v timeout -k 10 120 python tools/time_sort.py 32 40 2>/dev/null | tail -n 1)"
done; done
TAG=r05x ROUNDS=2 CONFIGS=$'base;RV_LIB_VARIANT=base;\ndefault;;\na256;RV_LIB_VARIANT=a256;' bash tools/gpu_bench_ab.sh
