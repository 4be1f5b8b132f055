# Per-kernel average durations (rocprofv3 --kernel-trace --stats over the
# eager per-conv profile, B=128 1080p) of two library builds, alternating:
#   TAG=x VARS="base default" KERNELS="sppf|decode" bash tools/gpu_kstats_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-kstats}; mkdir -p $O
i=0
for v in ${VARS:-base default base default}; do
  i=$((i + 1))
  RV_LIB_VARIANT=$v B=${B:-128} N=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o k -- python3 tools/conv_profile.py > $O/run_$i.log 2>&1 || exit 1
  f=$(find $O/p$i -name "*kernel_stats.csv" | head -n 1)
  cp $f $O/stats_${i}_$v.csv
  rm -rf $O/p$i
  echo "$v: $(python3 -c "
import csv
for r in csv.DictReader(open('$O/stats_${i}_$v.csv')):
    import re
    if re.search('${KERNELS:-sppf}', r['Name']): print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us avg;', end=' ')
")"
done
