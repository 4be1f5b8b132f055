#!/bin/bash
# Bench lines for a list of extra bench.py argument sets (one per line of
# $ARGS_FILE, or the ARGSETS env separated by ';').  Each run has its own
# time limit; the first failure ends the script.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sweep
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
i=0
for a in "${SETS[@]}"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-40} $a \
    > gpurun_out/sweep/b$i.json 2> gpurun_out/sweep/b$i.err
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/b$i.json')); print('$a ->', d['value'], d['ms_per_step'])"
  i=$((i+1))
done
