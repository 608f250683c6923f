#!/bin/bash
# stored propagators for blocks of 5..16 rows: tests, tunable-bus bench (blkp on / off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05v_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05v_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  QOC_BLKP=$v timeout -k 10 300 python bench.py --config tunable_bus --steps 5 --warmup 2 --no-cpu > gpurun_out/r05v_bench_tb$v.json 2> gpurun_out/r05v_bench_tb$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05v_bench_tb$v.json')); print('blkp=$v', round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms_per_launch'],3) for k, v in d['kernels'].items() if isinstance(v, dict) and 'ms_per_launch' in v})"
done
