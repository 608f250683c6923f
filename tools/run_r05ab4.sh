#!/bin/bash
# kernel trace of the tunable bus with one seed group (formation, then chains: no overlap) and with the default four
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for p in 1 4; do
  QOC_BLKP_PARTS=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ab4_p$p -o run -- python3 $R/bench.py --config tunable_bus --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/r05ab4_p$p.log 2>&1 || exit $?
done
