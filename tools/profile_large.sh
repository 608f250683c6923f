#!/bin/bash
# Profiling recipe for the large-N (synthetic) pipeline: kernel trace + stats, then separate PMC passes.
# Usage: tools/profile_large.sh <tag>
set -eo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}_synthetic_fused
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --config synthetic --steps 1 --warmup 1 --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- $B > "$OUT/bench_trace.json" 2> "$OUT/trace.log"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_bgemm --kernel-trace -d "$OUT/pmc_fetch" -o run -f csv -- $B > /dev/null 2> "$OUT/pmc_fetch.log"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_bgemm --kernel-trace -d "$OUT/pmc_write" -o run -f csv -- $B > /dev/null 2> "$OUT/pmc_write.log"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex k_bgemm --kernel-trace -d "$OUT/pmc_sq" -o run -f csv -- $B > /dev/null 2> "$OUT/pmc_sq.log"
echo "profile done: $OUT"
