#!/bin/bash
# 12-wave fused backward ($1: tag): focused tests ($2 over $3), then cavity benches over worker-wave counts.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04w}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${3:-tests} -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
for v in "" "QOC_BLKU_GFW=4" "QOC_BLKU_GFW=6" "QOC_BLKU_GFW=7" "QOC_BLKU_FW=6" "QOC_BLKU_FW=8"; do
  tag=${v:-default}
  env $v timeout -k 10 200 python bench.py --config cavity --no-cpu > gpurun_out/${T}_bench_cavity_${tag}.json 2> gpurun_out/${T}_bench_cavity_${tag}.err || exit 1
done
timeout -k 10 200 python bench.py --config zz_batch --no-cpu > gpurun_out/${T}_bench_zz_batch.json 2> gpurun_out/${T}_bench_zz_batch.err || exit 1
echo done
