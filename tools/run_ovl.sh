#!/bin/bash
# Backward-chain / gradient overlap A/B (QOC_BWD_CHUNKS, QOC_BWD_LAST) on cavity and zz, plus parity with it on.
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/ovl
mkdir -p $o
for cfg in cavity zz_batch; do
  for ch in 1 2 4 8; do
    QOC_BWD_CHUNKS=$ch timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_c$ch.json 2> $o/${cfg}_c$ch.err || exit 1
  done
  for lf in 0.5 0.25; do
    QOC_BWD_CHUNKS=4 QOC_BWD_LAST=$lf timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_c4_l$lf.json 2> $o/${cfg}_c4_l$lf.err || exit 1
  done
done
QOC_BWD_CHUNKS=4 QOC_BWD_LAST=0.5 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ode.py > $o/parity_c4.log 2>&1 || exit 1
echo done
