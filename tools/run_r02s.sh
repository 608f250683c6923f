#!/bin/bash
# Large-N T12 exponential: focused tests, full -m gpu suite, bench lines of every config, then the synthetic
# and tunable-bus profiles (each step time-limited; the script stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r02s}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_large_n.py > gpurun_out/${T}_focus.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1 || exit 1
for c in synthetic cavity zz_batch tunable_bus; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
./tools/profile_large.sh r02d || exit 1
./tools/profile.sh tunable_bus r02d || exit 1
echo done
