#!/bin/bash
# quaternion form: segmented tests, cavity/zz benches, probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkseg.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05u_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05u_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in cavity zz_batch; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/r05u_bench_$cfg.json 2> gpurun_out/r05u_bench_$cfg.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05u_bench_$cfg.json')); print('$cfg', round(d['value'],1), round(d['ms_per_step'],4), round(d['roofline']['ms_per_launch'],4), round(d['roofline']['frac'],3))"
done
timeout -k 10 120 ./tools/blkseg_probe 2 > gpurun_out/r05u_probe2.txt 2>&1; head -2 gpurun_out/r05u_probe2.txt
