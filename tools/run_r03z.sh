#!/bin/bash
# Round-3 check: full -m gpu suite, bench lines of every config (with the CPU baseline), smoke.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03z}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1 || exit 1
for c in cavity zz_batch tunable_bus synthetic; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err || exit 1
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo done
