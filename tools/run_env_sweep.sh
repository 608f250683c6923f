#!/bin/bash
# bench of one config under environment variants: tools/run_env_sweep.sh <tag> <config> <form> "VAR=v ..." ...
set -o pipefail
T=$1; CFG=$2; FORM=$3; shift 3
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --config $CFG --call-form $FORM --no-cpu --steps ${STEPS:-20} > gpurun_out/${T}_${CFG}_v$i.json 2> gpurun_out/${T}_${CFG}_v$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${T}_${CFG}_v$i.json')); r=d['roofline']; print('$CFG $FORM [$v]', round(d['value'],1), round(d['ms_per_step'],4), r['kernel'], round(r['ms_per_launch'],4), round(r['frac'],3))"
done
