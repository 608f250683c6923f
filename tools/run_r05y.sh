#!/bin/bash
# stored propagators: tests + tunable-bus bench (skew transposes, closed-form squarings)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05y_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config tunable_bus --steps 5 --warmup 2 --no-cpu > gpurun_out/r05y_bench_tb.json 2> gpurun_out/r05y_bench_tb.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r05y_bench_tb.json')); print(round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms_per_launch'],3) for k, v in d['kernels'].items() if isinstance(v, dict) and 'ms_per_launch' in v}, d['roofline']['kernel'], round(d['roofline']['frac'],3), d['kernels']['k_expm'].get('products_per_unit'))"
