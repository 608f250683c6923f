#!/bin/bash
# Stored propagators A/B ($1: tag): focused tests ($2 over $3), then cavity / zz benches with and without them.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04s}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${3:-tests} -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
for cfg in cavity zz_batch; do
  for v in "QOC_BLKU_STOREU=1" "QOC_BLKU_STOREU=0"; do
    env $v timeout -k 10 200 python bench.py --config $cfg --no-cpu > gpurun_out/${T}_bench_${cfg}_${v#*=}.json 2> gpurun_out/${T}_bench_${cfg}_${v#*=}.err || exit 1
  done
done
echo done
