#!/bin/bash
# round-6 closing measurements: kernel traces + PMC passes of the tunable bus (fused and split; the other configs'
# kernels did not change since r06p), then every config's bench lines (tools/run_r06_bench.sh).  Usage: <tag>
set -o pipefail
T=${1:-r06g}
for f in fused split; do
  STEPS=3 timeout -k 10 900 tools/profile.sh tunable_bus $T $f > gpurun_out/${T}_prof_tunable_bus_$f.log 2>&1 || exit 1
done
timeout -k 10 1000 tools/run_r06_bench.sh $T || exit 1
echo close done
