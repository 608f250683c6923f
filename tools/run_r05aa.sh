#!/bin/bash
# chain chunk size 8 vs 4 with seed groups
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05aa_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  QOC_BLKP_PRIO=$v timeout -k 10 300 python bench.py --config tunable_bus --steps 5 --warmup 2 --no-cpu > gpurun_out/r05aa_bench_prio$v.json 2> gpurun_out/r05aa_bench_prio$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05aa_bench_prio$v.json')); print('prio=$v', round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms_per_launch'],3) for k, v in d['kernels'].items() if isinstance(v, dict) and 'ms_per_launch' in v})"
done
