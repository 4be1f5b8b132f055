set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_graph_events.py > gpurun_out/r02_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -8 gpurun_out/r02_probe.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --conv-timing eager --tune-save gpurun_out/tune_r02b.json > gpurun_out/r02_bench2.json 2> gpurun_out/r02_bench2.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r02_bench2.err; cat gpurun_out/r02_bench2.json
exit $rc
