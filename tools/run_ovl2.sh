#!/bin/bash
# Overlap A/B 2: issue priority of the chain waves / gradient stream priority, chunk counts.
set -o pipefail
o=gpurun_out/ovl2
mkdir -p $o
for cfg in cavity zz_batch; do
  for pr in 0 1 2 3; do
    QOC_BWD_CHUNKS=4 QOC_BWD_LAST=0.5 QOC_BWD_PRIO=$pr timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_p$pr.json 2> $o/${cfg}_p$pr.err || exit 1
  done
  for ch in 3 6; do
    QOC_BWD_CHUNKS=$ch QOC_BWD_LAST=0.5 QOC_BWD_PRIO=1 timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_c${ch}_p1.json 2> $o/${cfg}_c${ch}_p1.err || exit 1
  done
done
echo done
