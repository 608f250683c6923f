#!/bin/bash
# kernel traces + PMC passes of the final round-6 build for the configs whose kernels changed after r06p / r06g
set -o pipefail
T=${1:-r06j}
for cf in "cavity fused" "zz_batch fused" "tunable_bus fused" "cavity split" "tunable_bus split"; do
  set -- $cf
  STEPS=3 timeout -k 10 900 tools/profile.sh $1 $T $2 > gpurun_out/${T}_prof_$1_$2.log 2>&1 || exit 1
done
echo profiles done
