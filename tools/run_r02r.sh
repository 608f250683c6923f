#!/bin/bash
# Round-2 check of the sandwich gradient (large-N) and the array-free Chebyshev prep: focused tests, the
# full -m gpu suite, then the synthetic / tunable-bus / cavity bench lines (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r02r}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_large_n.py > gpurun_out/${T}_focus.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1 || exit 1
for c in synthetic tunable_bus cavity; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
echo done
