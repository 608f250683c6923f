#!/bin/bash
# A/B of the overlapped backward's range split (QOC_BWD_CHUNKS ranges, last one QOC_BWD_LAST of a uniform one).
set -o pipefail
o=gpurun_out/sweep_bwd
mkdir -p $o
for cfg in cavity zz_batch; do
  for ch in 4 6 8; do
    for last in 0.25 0.5; do
      QOC_BWD_CHUNKS=$ch QOC_BWD_LAST=$last timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_c${ch}_l${last}.json 2> $o/${cfg}_c${ch}_l${last}.err || exit 1
    done
  done
done
echo done
