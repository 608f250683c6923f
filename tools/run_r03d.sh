#!/bin/bash
# Concurrent modes A/B on one box: QOC_CONCURRENT=0 (sequential captured backward), 2 (two streams), 1 (one dual
# launch, default); the concurrent tests first; then a kernel trace of the default on cavity.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03d}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_spline.py > gpurun_out/${T}_focus.log 2>&1 || exit 1
for c in cavity tunable_bus zz_batch; do
  for mode in 0 2 1; do
    QOC_CONCURRENT=$mode timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_c${mode}_$c.json 2> gpurun_out/${T}_c${mode}_$c.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace_cavity -o run -f csv -- python3 bench.py --config cavity --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_trace_cavity.json 2> gpurun_out/${T}_trace_cavity.err || exit 1
echo done
