#!/bin/bash
# round 5: full GPU check (pytest -m gpu, smoke), rocprofv3 profiles of cavity and zz, benches of every config.
# $1: tag.  Each GPU step time-limited; stops at the first failure.
set -o pipefail
T=${1:-r05x}
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
for cfg in cavity zz_batch; do
  STEPS=5 timeout -k 10 600 bash tools/profile.sh $cfg $T > gpurun_out/${T}_prof_$cfg.log 2>&1 || exit $?
done
for cfg in cavity zz_batch tunable_bus cavity_dense synthetic; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_$cfg.json')); print('$cfg', round(d['value'],1), round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['frac'],3), (d.get('parity_vs_cpu_port') or {}).get('max_abs_dJ'))"
done
