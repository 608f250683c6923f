#!/bin/bash
# tunable-bus bench under environment variants: tools/run_tb_sweep.sh <tag> "VAR=v VAR2=w" "VAR=x" ...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --config tunable_bus --no-cpu --steps 10 > gpurun_out/${T}_v$i.json 2> gpurun_out/${T}_v$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${T}_v$i.json')); k=d['kernels']; print('$v', round(d['value'],1), round(d['ms_per_step'],3), {n: round(k[n]['ms_per_launch'],3) for n in ('k_expm','k_chain_fwd','k_grad')})"
done
