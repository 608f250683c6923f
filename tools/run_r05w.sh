#!/bin/bash
# stored propagators: chunked LDS-DMA chains; formation occupancy 2 vs 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05w_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 3 2; do
  QOC_BLKP_OCC=$v timeout -k 10 300 python bench.py --config tunable_bus --steps 5 --warmup 2 --no-cpu > gpurun_out/r05w_bench_occ$v.json 2> gpurun_out/r05w_bench_occ$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05w_bench_occ$v.json')); print('occ=$v', round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms_per_launch'],3) for k, v in d['kernels'].items() if isinstance(v, dict) and 'ms_per_launch' in v})"
done
