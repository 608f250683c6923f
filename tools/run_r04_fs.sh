#!/bin/bash
# Forward prefix groups apart from the fused backward's (QOC_BLKU_FS=2) against none ($1: tag): block parity tests
# under FS=2, then cavity / zz benches under FS=1 and FS=2; each step time-limited, stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04fs}
K="prop or ((zz_batch or cavity) and full_size and auto) or costate or gradient_orders or fused_chunk"
F="tests/test_gpu_blk.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py"
QOC_BLKU_FS=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $F -k "$K" > gpurun_out/${T}_focus2.log 2>&1 || exit 1
for f in 2 1; do
  for cfg in cavity zz_batch; do
    QOC_BLKU_FS=$f timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/${T}_f${f}_$cfg.json 2> gpurun_out/${T}_f${f}_$cfg.err || exit 1
  done
done
echo done
