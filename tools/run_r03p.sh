#!/bin/bash
# Per-term slope of the block chains (Chebyshev vs Taylor terms on the same build), then final-code profiles.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03p}
for c in cavity zz_batch; do
  QOC_TCHAIN_POLY=taylor timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_taylor_$c.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/${T}_cheb_$c.json 2>/dev/null || exit 1
done
for c in cavity zz_batch tunable_bus; do
  ./tools/profile.sh $c $T > gpurun_out/${T}_prof_$c.log 2>&1 || exit 1
done
echo done
