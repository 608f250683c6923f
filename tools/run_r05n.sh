#!/bin/bash
# tunable bus: split accumulators (tests + bench), block-propagator measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blk.py -k "tunable or dead or mfma" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05n_tests.log; [ $rc -eq 0 ] || exit $rc
sum() { python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],3), {a:round(b.get('ms_per_launch',0),3) if isinstance(b,dict) else b for a,b in k.items()})" "$1" "$2"; }
timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05n_tb.json 2> gpurun_out/r05n_tb.err || exit $?
sum gpurun_out/r05n_tb.json tunable_bus
timeout -k 10 500 python tools/tb_blockprop.py 5 > gpurun_out/r05n_tb_blockprop.txt 2>&1; rc=$?; cat gpurun_out/r05n_tb_blockprop.txt | tail -4; exit $rc
