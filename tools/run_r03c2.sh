#!/bin/bash
# Block tests, then Chebyshev (default) and Taylor bench lines of the block configs on the same build
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03c2}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_blk.py > gpurun_out/${T}_blk.log 2>&1 || exit 1
for c in cavity zz_batch tunable_bus; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_cheb_$c.json 2>/dev/null || exit 1
  QOC_TCHAIN_POLY=taylor timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_taylor_$c.json 2>/dev/null || exit 1
done
echo done
