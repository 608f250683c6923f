#!/bin/bash
# Round-4 full GPU check ($1: tag): the whole -m gpu suite, smoke(), then the bench of every config (cavity with
# its cpu_baseline leg); each step time-limited; the call ends at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04full}
timeout -k 10 1500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench_cavity.json 2> gpurun_out/${T}_bench_cavity.err || exit 1
for cfg in ${2:-zz_batch cavity_dense tunable_bus synthetic}; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.err || exit 1
done
echo done
