#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03q}
true
true
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rot.py tests/test_gpu_concurrent.py tests/test_gpu_parity.py > gpurun_out/${T}_test.log 2>&1 || exit 1
for c in zz_batch tunable_bus cavity; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_$c.json 2>gpurun_out/${T}_$c.err || exit 1
done
echo done
