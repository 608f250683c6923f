#!/bin/bash
# Remaining GPU tests after a fix (pytest -k $2) and bench lines of the chain configs.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_spline.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py > gpurun_out/${T}_gputest.log 2>&1 || exit 1
for c in cavity zz_batch tunable_bus; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
echo done
