#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03j}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rot.py tests/test_gpu_concurrent.py tests/test_gpu_parity.py > gpurun_out/${T}_test.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config zz_batch --no-cpu > gpurun_out/${T}_zz.json 2>gpurun_out/${T}_zz.err || exit 1
timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/${T}_tb.json 2>gpurun_out/${T}_tb.err || exit 1
QOC_TCHAIN_ROT=3 timeout -k 10 300 python bench.py --config cavity --no-cpu > gpurun_out/${T}_cav3.json 2>gpurun_out/${T}_cav3.err || exit 1
timeout -k 10 300 python bench.py --config cavity --no-cpu > gpurun_out/${T}_cav.json 2>gpurun_out/${T}_cav.err || exit 1
echo done
