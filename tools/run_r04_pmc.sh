#!/bin/bash
# SQ counters of the block-propagator kernels on the cavity and zz benches ($1: tag), one rocprofv3 pass each,
# plus the probe's segment breakdown; each step time-limited, stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04pmc}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 tools/blku_probe 2 > gpurun_out/${T}_probe2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for cfg in cavity zz_batch; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/${T}_pmc_$cfg -o pmc -- python3 $R/bench.py --config $cfg --no-cpu --steps 3 --warmup 1 > $R/gpurun_out/${T}_pmc_$cfg.log 2>&1 || exit 1
done
echo done
