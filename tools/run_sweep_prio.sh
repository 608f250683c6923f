#!/bin/bash
# Chain-wave priority / low-priority gradient stream A/B with the state-side pass (QOC_BWD_PRIO), two repeats.
set -o pipefail
o=gpurun_out/sweep_prio
mkdir -p $o
for rep in 1 2; do
  for cfg in cavity zz_batch; do
    for pr in 0 1 2 3; do
      QOC_BWD_PRIO=$pr timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_p${pr}_r${rep}.json 2> $o/${cfg}_p${pr}_r${rep}.err || exit 1
    done
  done
done
echo done
