#!/bin/bash
# Concurrent modes A/B (QOC_CONCURRENT=0 / 2 / 1) on the chain configs, the large-N tests and synthetic bench with the
# T8 / 2-norm exponential, then a kernel trace of the default cavity bench.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03e}
export TMPDIR=/tmp
timeout -k 10 60 tools/mfma4_lat > gpurun_out/${T}_mfma4_lat.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_spline.py tests/test_gpu_large_n.py > gpurun_out/${T}_focus.log 2>&1 || exit 1
for c in cavity tunable_bus zz_batch; do
  for mode in 0 2 1; do
    QOC_CONCURRENT=$mode timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_c${mode}_$c.json 2> gpurun_out/${T}_c${mode}_$c.err || exit 1
  done
done
timeout -k 10 300 python bench.py --config synthetic --no-cpu > gpurun_out/${T}_synthetic.json 2> gpurun_out/${T}_synthetic.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace_cavity -o run -f csv -- python3 bench.py --config cavity --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_trace_cavity.json 2> gpurun_out/${T}_trace_cavity.err || exit 1
echo done
