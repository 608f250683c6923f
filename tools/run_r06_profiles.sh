#!/bin/bash
# round-6 profiles: kernel trace + FETCH / WRITE / SQ passes of every config (tools/profile.sh), the split call form
# of cavity and the tunable bus, and the instruction-mix passes of the segmented eval (tools/profile_mix.sh)
set -o pipefail
T=${1:-r06}
for cfg in cavity zz_batch tunable_bus cavity_dense; do
  STEPS=3 timeout -k 10 900 tools/profile.sh $cfg $T fused > gpurun_out/${T}_prof_$cfg.log 2>&1 || exit 1
done
for cfg in cavity tunable_bus; do
  STEPS=3 timeout -k 10 900 tools/profile.sh $cfg $T split > gpurun_out/${T}_prof_${cfg}_split.log 2>&1 || exit 1
done
timeout -k 10 900 tools/profile_large.sh $T > gpurun_out/${T}_prof_synthetic.log 2>&1 || exit 1
echo profiles done
