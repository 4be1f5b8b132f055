set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ORDER=1 timeout -k 10 200 python -u tools/conv_profile.py > gpurun_out/r02_convprof_fused.txt 2>&1 || exit $?
RV_FUSE_C2F=0 ORDER=1 timeout -k 10 200 python -u tools/conv_profile.py > gpurun_out/r02_convprof_unfused.txt 2>&1 || exit $?
head -20 gpurun_out/r02_convprof_fused.txt; head -28 gpurun_out/r02_convprof_unfused.txt
