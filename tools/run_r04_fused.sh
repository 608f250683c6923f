#!/bin/bash
# Fused block backward: focused parity tests ($2 over $3), then cavity / zz benches over worker-wave counts, chunk
# sizes and prefix groups (env overrides of blku_shape); each step time-limited, stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04f}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${3:-tests} -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
for cfg in cavity zz_batch; do
  for v in "" "QOC_BLKU_GFW=3" "QOC_BLKU_GFW=5" "QOC_BLKU_GFW=7" "QOC_BLKU_GC=8" "QOC_BLKU_GC=32" "QOC_BLKU_S=2" "QOC_BLKU_FW=3" "QOC_BLKU_FW=6" "QOC_BLKU_C=16" "QOC_BLKU_FUSED=0"; do
    tag=${v:-default}
    env $v timeout -k 10 120 python bench.py --config $cfg --no-cpu --steps 10 > gpurun_out/${T}_bench_${cfg}_${tag}.json 2> gpurun_out/${T}_bench_${cfg}_${tag}.err || exit 1
  done
done
echo done
