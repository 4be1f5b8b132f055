# config-2 call anatomy (tools/c2_host.py) under variants, alternating:
#   TAG=x VARIANTS="base;RV_LIB_VARIANT=base|new;" bash tools/gpu_c2_host.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c2h}; mkdir -p $O
IFS='|' read -ra VS <<< "${VARIANTS:-base;}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    name=${v%%;*}; envs=${v#*;}
    env NAME=$name $envs timeout -k 10 200 python3 tools/c2_host.py 2>> $O/err.txt | tee -a $O/out.txt || exit $?
  done
done
