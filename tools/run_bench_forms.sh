#!/bin/bash
# bench lines of one config in each call form (tools/run_bench_forms.sh <tag> <config> [forms...]): fused
# (qoc_eval_dev), split (qoc_propagate_dev + qoc_grape_sensitivity_dev), ipopt (the spline callbacks, host arrays)
set -o pipefail
T=${1:-r06}; CFG=${2:-cavity}; shift 2
FORMS=${@:-fused split ipopt}
mkdir -p gpurun_out
for f in $FORMS; do
  timeout -k 10 300 python bench.py --config $CFG --call-form $f --no-cpu --steps ${STEPS:-20} --warmup ${WARMUP:-3} \
    > gpurun_out/${T}_${CFG}_${f}.json 2> gpurun_out/${T}_${CFG}_${f}.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/${T}_${CFG}_${f}.json')); print('$CFG $f', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done
