#!/bin/bash
# same-box A/B of the bench between build_ab/prev (a previous commit's build) and the working tree, alternating.
# $1: config, $2: repeats, $3: tag
set -o pipefail
CFG=${1:-cavity}; REP=${2:-3}; T=${3:-ab}
mkdir -p gpurun_out
for rep in $(seq 1 $REP); do
  (cd build_ab/prev && timeout -k 10 300 python bench.py --config $CFG --no-cpu > ../../gpurun_out/${T}_prev_$rep.json 2> ../../gpurun_out/${T}_prev_$rep.err) || exit $?
  timeout -k 10 300 python bench.py --config $CFG --no-cpu > gpurun_out/${T}_head_$rep.json 2> gpurun_out/${T}_head_$rep.err || exit $?
  python -c "import json; a=json.load(open('gpurun_out/${T}_prev_$rep.json')); b=json.load(open('gpurun_out/${T}_head_$rep.json')); print('$CFG prev', round(a['value'],1), round(a['roofline']['ms_per_launch'],4), ' head', round(b['value'],1), round(b['roofline']['ms_per_launch'],4))"
done
