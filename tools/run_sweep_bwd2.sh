#!/bin/bash
# Range split A/B with the state-side pass on (QOC_BWD_CHUNKS x QOC_BWD_LAST), two alternating repeats.
set -o pipefail
o=gpurun_out/sweep_bwd2
mkdir -p $o
for rep in 1 2; do
  for cfg in cavity zz_batch; do
    for ch in 3 4 5; do
      for last in 0.5 0.75; do
        QOC_BWD_CHUNKS=$ch QOC_BWD_LAST=$last timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_c${ch}_l${last}_r${rep}.json 2> $o/${cfg}_c${ch}_l${last}_r${rep}.err || exit 1
      done
    done
  done
done
for rep in 1 2; do
  for pre in 0 1; do
    QOC_BWD_PRESTATE=$pre timeout -k 10 120 python -u bench.py --config tunable_bus --steps 10 --warmup 2 --no-cpu > $o/tunable_bus_p${pre}_r${rep}.json 2> $o/tunable_bus_p${pre}_r${rep}.err || exit 1
  done
done
echo done
