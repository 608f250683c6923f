#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   1. kernel trace + stats of bench.py (per-kernel average duration)
#   2. PMC passes (separate runs, --kernel-trace only): FETCH_SIZE, WRITE_SIZE, MFMA/VALU activity
# Usage: tools/profile.sh <config> <tag>
set -eo pipefail
CFG=${1:-cavity}
TAG=${2:-r01}
FORM=${3:-fused}   # bench.py --call-form
OUT=gpurun_out/prof_${TAG}_${CFG}_${FORM}
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-3}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- \
  python3 bench.py --config "$CFG" --call-form $FORM --steps $STEPS --warmup 1 --no-cpu --side "" > "$OUT/bench_trace.json" 2> "$OUT/trace.log"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run -f csv -- \
  python3 bench.py --config "$CFG" --call-form $FORM --steps $STEPS --warmup 1 --no-cpu --side "" > /dev/null 2> "$OUT/pmc_fetch.log"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run -f csv -- \
  python3 bench.py --config "$CFG" --call-form $FORM --steps $STEPS --warmup 1 --no-cpu --side "" > /dev/null 2> "$OUT/pmc_write.log"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES --kernel-trace -d "$OUT/pmc_sq" -o run -f csv -- \
  python3 bench.py --config "$CFG" --call-form $FORM --steps $STEPS --warmup 1 --no-cpu --side "" > /dev/null 2> "$OUT/pmc_sq.log" || true
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmc_sq2" -o run -f csv -- \
  python3 bench.py --config "$CFG" --call-form $FORM --steps $STEPS --warmup 1 --no-cpu --side "" > /dev/null 2> "$OUT/pmc_sq2.log" || true
echo "profile done: $OUT"
