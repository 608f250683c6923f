#!/bin/bash
# tunable bus: dead-block tests, then A/B of Chebyshev prep variants / dead-block skipping against the round-3 build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blk.py -k "tunable or dead" tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_tests.log; [ $rc -eq 0 ] || exit $rc
sum() { python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],3), d.get('parity',{}), {a:round(b.get('ms_per_launch',0),3) if isinstance(b,dict) else b for a,b in k.items()})" "$1" "$2"; }
for rep in 1 2; do
  (cd build_ab/r03 && timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > ../../gpurun_out/r05k_r03_$rep.json 2> ../../gpurun_out/r05k_r03_$rep.err) || exit $?
  sum gpurun_out/r05k_r03_$rep.json r03
  for v in "QOC_BLK_DEAD=1" "QOC_BLK_DEAD=0" "QOC_TCHEB_PREP=0 QOC_BLK_DEAD=0" "QOC_TCHEB_PW=64 QOC_BLK_DEAD=0" "QOC_TCHEB_PREP=0 QOC_BLK_DEAD=1"; do
    tag=$(echo $v | tr ' =' '__')
    env $v timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05k_${tag}_$rep.json 2> gpurun_out/r05k_${tag}_$rep.err || exit $?
    sum gpurun_out/r05k_${tag}_$rep.json "$tag"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_n.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k_largen.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_largen.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config synthetic --no-cpu > gpurun_out/r05k_synthetic.json 2> gpurun_out/r05k_synthetic.err || exit $?
sum gpurun_out/r05k_synthetic.json synthetic
timeout -k 10 120 ./tools/bgemm_bench 256 1260 > gpurun_out/r05k_bgemm_bench.txt 2>&1 && cat gpurun_out/r05k_bgemm_bench.txt
