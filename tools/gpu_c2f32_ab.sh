set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c32; mkdir -p $O
for r in 1 2; do
  B=128 timeout -k 10 300 python -u tools/conv_profile.py > $O/unf_$r.log 2>&1 || exit 1
  RV_FUSE_C2F32=1 B=128 timeout -k 10 300 python -u tools/conv_profile.py > $O/fus_$r.log 2>&1 || exit 1
  echo "r$r unfused: $(grep 'conv sum' $O/unf_$r.log)"; echo "r$r fused32: $(grep 'conv sum' $O/fus_$r.log)"
done
