#!/bin/bash
# Block tests + bench lines of cavity, zz, tunable bus (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03v}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_blk.py > gpurun_out/${T}_blk.log 2>&1 || exit 1
for c in cavity zz_batch tunable_bus; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_$c.json 2>gpurun_out/${T}_$c.err || exit 1
done
echo done
