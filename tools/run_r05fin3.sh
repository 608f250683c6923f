#!/bin/bash
# round 5 last closing check: pytest -m gpu, smoke, the tunable-bus bench with the CPU baseline.  $1: tag
set -o pipefail
T=${1:-r05fin3}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python bench.py --config tunable_bus > gpurun_out/${T}_bench_tunable_bus.json 2> gpurun_out/${T}_bench_tunable_bus.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_tunable_bus.json')); print('tunable_bus', round(d['value'],1), round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['frac'],3), d['roofline']['traffic'], (d.get('parity_vs_cpu_port') or {}).get('max_abs_dJ'))"
