#!/bin/bash
# Round-3 profiles: rocprofv3 kernel trace + PMC passes of every config (tools/profile.sh, profile_large.sh)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03u}
for c in cavity zz_batch tunable_bus; do
  ./tools/profile.sh $c $T > gpurun_out/${T}_prof_$c.log 2>&1 || exit 1
done
./tools/profile_large.sh $T > gpurun_out/${T}_prof_synthetic.log 2>&1 || exit 1
echo done
