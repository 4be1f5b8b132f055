# config-2 latency under environment variants, alternating:
#   TAG=x VARIANTS="base;RV_FUSE_C2F32=1|heads0;RV_HEAD_STREAMS=0" ROUNDS=2 bash tools/gpu_c2_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c2ab}; mkdir -p $O
IFS='|' read -ra VS <<< "${VARIANTS:-base;}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    name=${v%%;*}; envs=${v#*;}
    env $envs timeout -k 10 200 python3 tools/bench_config2.py --cpu-frames 0 --iters ${ITERS:-300} > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    echo "$name r$r: $(python3 -c "import json,sys; d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]); L=d['latency']; print(d['value'], L['forward_native']['median_ms'], d['device_ms_back_to_back'])")"
  done
done
