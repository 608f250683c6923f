#!/bin/bash
# PMC passes on the standalone batched-GEMM microbenchmark (tools/bgemm_bench.hip) at the synthetic
# shape (N = 256, 1260 items = one chunk).  Separate passes: TCC FETCH_SIZE, TCC WRITE_SIZE, SQ.
set -eo pipefail
OUT=gpurun_out/prof_${1:-r01}_bgemm
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="256 1260"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- ./tools/bgemm_bench $ARGS > "$OUT/bench.txt" 2> "$OUT/trace.log"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run -f csv -- ./tools/bgemm_bench $ARGS > /dev/null 2> "$OUT/pmc_fetch.log"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run -f csv -- ./tools/bgemm_bench $ARGS > /dev/null 2> "$OUT/pmc_write.log"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d "$OUT/pmc_sq" -o run -f csv -- ./tools/bgemm_bench $ARGS > /dev/null 2> "$OUT/pmc_sq.log"
echo "profile done: $OUT"
