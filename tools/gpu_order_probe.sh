# Does a preceding GPU test suite change the bench? bench, the -m gpu suite,
# bench, bench (each bench autotunes in-process, as the driver's does)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-order}; mkdir -p $O
B="python -u bench.py --steps 20 --no-secondary --no-cpu-baseline --conv-timing none"
timeout -k 10 300 $B > $O/b1.json 2> $O/b1.err || exit 1
echo "fresh: $(python3 -c "import json;d=json.load(open('$O/b1.json'));print(d['value'], (d.get('device_only') or {}).get('value'), d.get('steady_state_frames_per_s'))")"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 20 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for i in 2 3; do
  timeout -k 10 300 $B > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "after tests #$i: $(python3 -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'], (d.get('device_only') or {}).get('value'), d.get('steady_state_frames_per_s'))")"
done
