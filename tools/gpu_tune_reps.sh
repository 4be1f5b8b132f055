# Autotuner repetitions per candidate (RV_AUTOTUNE_REPS) vs the bench, each
# run tuning in-process as the driver's does, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-tunereps}; mkdir -p $O
B="python -u bench.py --steps 20 --no-secondary --no-cpu-baseline --conv-timing none"
for r in 1 2; do for reps in 10 25; do
  RV_AUTOTUNE_REPS=$reps timeout -k 10 400 $B > $O/r${reps}_$r.json 2> $O/r${reps}_$r.err || exit 1
  echo "reps $reps #$r: $(python3 -c "import json;d=json.load(open('$O/r${reps}_$r.json'));print(d['value'], (d.get('device_only') or {}).get('value'), d.get('steady_state_frames_per_s'))")"
done; done
