#!/bin/bash
# closing bench lines of round 6: every config in the fused form with its CPU baseline, then the split and ipopt call
# forms (no CPU leg), and the B = 1 zz plumbing latency in each form.  tools/run_r06_bench.sh <tag>
set -o pipefail
T=${1:-r06f}
mkdir -p gpurun_out
run() {  # run <file stem> <bench args...>
  local f=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/${T}_$f.json 2> gpurun_out/${T}_$f.err || { echo "FAILED $f"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$f.json')); c=d.get('cpu_baseline') or {}; p=d.get('parity_vs_cpu_port') or {}; print('$f', round(d['value'],2), 'ms/step', round(d['ms_per_step'],4), d['roofline'].get('kernel'), round(d['roofline']['frac'],3), 'cpu', c.get('value'), 'dJ', p.get('max_abs_dJ'))"
}
run cavity_fused --config cavity --steps 20 --warmup 3 --side ''
for c in zz_batch tunable_bus cavity_dense; do run ${c}_fused --config $c --steps 20 --warmup 3; done
run synthetic_fused --config synthetic --steps 2 --warmup 1
for c in cavity zz_batch tunable_bus; do
  for f in split ipopt; do run ${c}_$f --config $c --call-form $f --steps 20 --warmup 3 --no-cpu; done
done
for f in fused split ipopt; do run zz_plumbing_$f --config zz_plumbing --call-form $f --steps 200 --warmup 20 --no-cpu; done
echo bench done
