#!/bin/bash
# k_bgemm_glds after the row-clamp fix: probe, microbench, large-N tests, synthetic bench (glds on / off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/glds_probe > gpurun_out/r05m_probe.txt 2>&1; rc=$?; grep -c "first bad" gpurun_out/r05m_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/bgemm_bench 256 1260 > gpurun_out/r05m_bgemm_bench.txt 2>&1; rc=$?
cat gpurun_out/r05m_bgemm_bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05m_largen.log 2>&1
rc=$?; tail -3 gpurun_out/r05m_largen.log; [ $rc -eq 0 ] || exit $rc
sum() { python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[2], round(d['value'],2), round(d['ms_per_step'],1), round(d['roofline']['frac'],3), {a:round(b.get('ms_per_launch',0),1) if isinstance(b,dict) else b for a,b in k.items()})" "$1" "$2"; }
timeout -k 10 600 python bench.py --config synthetic --no-cpu > gpurun_out/r05m_synthetic.json 2> gpurun_out/r05m_synthetic.err || exit $?
sum gpurun_out/r05m_synthetic.json synthetic_glds
QOC_BGEMM_GLDS=0 timeout -k 10 600 python bench.py --config synthetic --no-cpu > gpurun_out/r05m_synthetic_off.json 2> gpurun_out/r05m_synthetic_off.err || exit $?
sum gpurun_out/r05m_synthetic_off.json synthetic_old
