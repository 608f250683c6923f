#!/bin/bash
# Round-3 GPU check: the new tests first, the full -m gpu suite, then bench lines of the chain configs.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03b}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrent.py > gpurun_out/${T}_focus.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1 || exit 1
for c in cavity zz_batch tunable_bus; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
echo done
