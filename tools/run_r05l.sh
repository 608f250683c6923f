#!/bin/bash
# k_bgemm_glds: microbench + variant cross-checks, the fp32 synthetic test with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bgemm_bench 256 1260 > gpurun_out/r05l_bgemm_bench.txt 2>&1; rc=$?
cat gpurun_out/r05l_bgemm_bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/bgemm_bench 256 64 768 > gpurun_out/r05l_bgemm_bench_k768.txt 2>&1; rc=$?
cat gpurun_out/r05l_bgemm_bench_k768.txt; [ $rc -eq 0 ] || exit $rc
QOC_BGEMM_GLDS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_large_n.py -x -q -k synthetic_n256_fp32 --timeout 200 --timeout-method thread > gpurun_out/r05l_off.log 2>&1; tail -2 gpurun_out/r05l_off.log
