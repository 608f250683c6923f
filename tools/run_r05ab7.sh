#!/bin/bash
# stored-propagator knobs re-checked after the trims (same box, 2 runs each)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for kv in "X=0" "QOC_BLKP_OCC=2" "QOC_BLKP_PRIO=1" "QOC_BLKP_CH=2" "QOC_BLKP_CH=8" "QOC_BLKP_PARTS=3" "QOC_BLKP_PARTS=6"; do
    t=${kv//=/_}
    env $kv timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05ab7_${t}_$rep.json 2> gpurun_out/r05ab7_${t}_$rep.err || exit $?
    python -c "import json; a=json.load(open('gpurun_out/r05ab7_${t}_$rep.json')); print('$kv', round(a['value'],1))"
  done
done
