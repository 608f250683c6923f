#!/bin/bash
# Instruction-mix PMC passes of one config (tools/profile_mix.sh <config> <tag> [call-form]): separate rocprofv3 runs,
# --kernel-trace only, <= 8 SQ counters each.  Summaries: python tools/pmc_db.py <dir>/pmc_*/.../*_results.db
set -eo pipefail
CFG=${1:-cavity}; TAG=${2:-r06}; FORM=${3:-fused}
OUT=gpurun_out/mix_${TAG}_${CFG}_${FORM}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --config $CFG --call-form $FORM --steps 3 --warmup 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
  SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d "$OUT/pmc_a" -o run -f csv -- $B \
  > /dev/null 2> "$OUT/a.log"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH \
  SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmc_b" -o run -f csv -- $B \
  > /dev/null 2> "$OUT/b.log"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY \
  SQ_WAIT_ANY SQ_WAVES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS --kernel-trace -d "$OUT/pmc_c" -o run -f csv -- $B \
  > /dev/null 2> "$OUT/c.log"
echo "mix done: $OUT"
