#!/bin/bash
# round 5 closing check, part A: pytest -m gpu, smoke, benches of every config (with the CPU baseline).  $1: tag
set -o pipefail
T=${1:-r05r}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
for cfg in cavity zz_batch tunable_bus cavity_dense synthetic; do
  timeout -k 10 400 python bench.py --config $cfg > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_$cfg.json')); print('$cfg', round(d['value'],1), round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['frac'],3), (d.get('parity_vs_cpu_port') or {}).get('max_abs_dJ'), d['cpu_baseline']['value'])"
done
