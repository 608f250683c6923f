#!/bin/bash
# Last-range fraction A/B with the state-side pass (QOC_BWD_LAST), two alternating repeats.
set -o pipefail
o=gpurun_out/sweep_last
mkdir -p $o
for rep in 1 2; do
  for cfg in cavity zz_batch; do
    for last in 0.3 0.4 0.5 0.6; do
      QOC_BWD_LAST=$last timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_l${last}_r${rep}.json 2> $o/${cfg}_l${last}_r${rep}.err || exit 1
    done
  done
done
echo done
