set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 120 "$@" > gpurun_out/probe_lanes.log 2>&1; rc=$?; grep -E "built|match|Error|error" gpurun_out/probe_lanes.log | head -5; echo "rc=$rc"; return $rc; }
run python -u tools/probe_lanes.py 0 2 8 || exit $?
run python -u tools/probe_lanes.py 1 2 8 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --conv-timing none --tune-save gpurun_out/tune6.json > gpurun_out/r02_b6_l1.json 2> gpurun_out/r02_b6_l1.err || exit $?
for L in 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --conv-timing none --tune-load gpurun_out/tune6.json --lanes $L > gpurun_out/r02_b6_l$L.json 2> gpurun_out/r02_b6_l$L.err || exit $?
done
for f in gpurun_out/r02_b6_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['sort'])"; done
