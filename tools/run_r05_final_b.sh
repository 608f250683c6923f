#!/bin/bash
# round 5 closing check, part B: rocprofv3 kernel traces + PMC passes (tools/profile.sh) of every config.  $1: tag
set -o pipefail
T=${1:-r05r}
mkdir -p gpurun_out
for cfg in cavity zz_batch tunable_bus synthetic cavity_dense; do
  STEPS=3 timeout -k 10 900 bash tools/profile.sh $cfg $T > gpurun_out/${T}_prof_$cfg.log 2>&1 || exit $?
  echo "$cfg profiled"
done
