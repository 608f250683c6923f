#!/bin/bash
# Round-2 check: k_bgemm swizzle A/B + bank-conflict PMC, new compress / z-cal tests, full GPU suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/bgemm_bench_old 256 1260 > gpurun_out/r02k_bgemm_old.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/bgemm_bench 256 1260 > gpurun_out/r02k_bgemm_new.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/r02k_pmc_new -o run -f csv -- ./tools/bgemm_bench 256 1260 > /dev/null 2> gpurun_out/r02k_pmc_new.log || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/r02k_pmc_old -o run -f csv -- ./tools/bgemm_bench_old 256 1260 > /dev/null 2> gpurun_out/r02k_pmc_old.log || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_compress.py tests/test_gpu_parity.py -k "zcal or compress or Compress" > gpurun_out/r02k_new.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02k_gputest.log 2>&1 || exit 1
echo done
