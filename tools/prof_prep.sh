set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in default np old; do
  RV_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_$v -o k -- python3 tools/time_preprocess.py > gpurun_out/pp_$v.log 2>&1
  find gpurun_out/pp_$v -name "*kernel_stats.csv" -exec cp {} gpurun_out/pp_${v}_stats.csv \;
done
