#!/bin/bash
# k_form_norm2 (generators in registers): large-N tests, synthetic bench; tunable-bus bench (live-block accounting)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05s_largen.log 2>&1
rc=$?; tail -2 gpurun_out/r05s_largen.log; [ $rc -eq 0 ] || exit $rc
sum() { python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[2], round(d['value'],2), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {a:round(b.get('ms_per_launch',0),2) if isinstance(b,dict) else b for a,b in k.items()})" "$1" "$2"; }
timeout -k 10 600 python bench.py --config synthetic --no-cpu > gpurun_out/r05s_synthetic.json 2> gpurun_out/r05s_synthetic.err || exit $?
sum gpurun_out/r05s_synthetic.json synthetic
timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05s_tb.json 2> gpurun_out/r05s_tb.err || exit $?
sum gpurun_out/r05s_tb.json tunable_bus
