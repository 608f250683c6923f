#!/bin/bash
# probe + SQ instruction counters of the segmented eval (probe binary, NB=2 cavity shape)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/blkseg_probe 2 > gpurun_out/r05e_probe.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/blkseg_probe 3 >> gpurun_out/r05e_probe.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/r05e_pmc -o pmc -- $R/tools/blkseg_probe 2 > $R/gpurun_out/r05e_pmc.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 -d $R/gpurun_out/r05e_pmc2 -o pmc -- $R/tools/blkseg_probe 2 > $R/gpurun_out/r05e_pmc2.log 2>&1
echo rc2=$?
cat $R/gpurun_out/r05e_probe.txt
