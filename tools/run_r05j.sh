#!/bin/bash
# segmented eval tests + benches, tunable-bus A/B (round-3 build vs HEAD), phase probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkseg.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05j_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in cavity zz_batch; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/r05j_bench_$cfg.json 2> gpurun_out/r05j_bench_$cfg.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05j_bench_$cfg.json')); print('$cfg', round(d['value'],1), round(d['ms_per_step'],4), round(d['roofline']['ms_per_launch'],4), round(d['roofline']['frac'],3))"
done
for rep in 1 2; do
  (cd build_ab/r03 && timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > ../../gpurun_out/r05j_tb_r03_$rep.json 2> ../../gpurun_out/r05j_tb_r03_$rep.err) || exit $?
  timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05j_tb_head_$rep.json 2> gpurun_out/r05j_tb_head_$rep.err || exit $?
  python -c "import json; a=json.load(open('gpurun_out/r05j_tb_r03_$rep.json')); b=json.load(open('gpurun_out/r05j_tb_head_$rep.json')); print('tunable_bus r03', round(a['value'],1), round(a['ms_per_step'],4), 'head', round(b['value'],1), round(b['ms_per_step'],4))"
done
timeout -k 10 120 ./tools/blkseg_probe 2 > gpurun_out/r05j_probe2.txt 2>&1 && timeout -k 10 120 ./tools/blkseg_probe 3 > gpurun_out/r05j_probe3.txt 2>&1
cat gpurun_out/r05j_probe2.txt gpurun_out/r05j_probe3.txt
