#!/bin/bash
# dead-row zeroing skipped when clean: block tests, tunable-bus bench, profile trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blk.py -k "tunable or dead or mfma" tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05t_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05t_tb.json 2> gpurun_out/r05t_tb.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r05t_tb.json')); print('tunable_bus', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))"
