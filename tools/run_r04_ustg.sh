#!/bin/bash
# Single staging wave for records + x_k + stored propagators (QOC_BLKU_USTG=1) against two ($1: tag): block parity
# tests under both, then cavity / zz benches under both; each step time-limited, stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04u}
K="prop or ((zz_batch or cavity) and full_size and auto) or costate or gradient_orders"
F="tests/test_gpu_blk.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py"
QOC_BLKU_USTG=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $F -k "$K" > gpurun_out/${T}_focus1.log 2>&1 || exit 1
for u in 1 2; do
  for cfg in cavity zz_batch; do
    QOC_BLKU_USTG=$u timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/${T}_u${u}_$cfg.json 2> gpurun_out/${T}_u${u}_$cfg.err || exit 1
  done
done
echo done
