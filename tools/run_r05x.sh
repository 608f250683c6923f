#!/bin/bash
# tunable bus on stored propagators: bench + rocprofv3 trace and PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config tunable_bus --steps 5 --warmup 2 --no-cpu > gpurun_out/r05x_bench_tb.json 2> gpurun_out/r05x_bench_tb.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r05x_bench_tb.json')); print(round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['ms_per_launch'],3) for k, v in d['kernels'].items() if isinstance(v, dict) and 'ms_per_launch' in v}, d['roofline']['kernel'], round(d['roofline']['frac'],3))"
STEPS=3 timeout -k 10 900 bash tools/profile.sh tunable_bus r05x > gpurun_out/r05x_prof.log 2>&1 || exit $?
echo profiled
