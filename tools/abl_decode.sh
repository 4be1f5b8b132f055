cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 32; do
RV_DECODE_ABLATE=$a N=5 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abl$a -o fwd -- python3 tools/trace_forward.py > gpurun_out/abl$a.log 2>&1
python3 tools/sweep_table.py --dump gpurun_out/abl$a > gpurun_out/abl$a.txt; rm -rf gpurun_out/abl$a
tail -1 gpurun_out/abl$a.txt
done
