#!/bin/bash
# blkp tests + the full-size device eval, then same-box A/B: prev, head, head with equal groups (QOC_BLKP_TAIL=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkp.py "tests/test_gpu_fullsize.py::test_tunable_bus_full_size_device_eval" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab6_t.log 2>&1 || { tail -20 gpurun_out/r05ab6_t.log; exit 1; }
tail -1 gpurun_out/r05ab6_t.log
for rep in 1 2 3; do
  (cd build_ab/prev && timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > ../../gpurun_out/r05ab6_prev_$rep.json 2> ../../gpurun_out/r05ab6_prev_$rep.err) || exit $?
  timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05ab6_head_$rep.json 2> gpurun_out/r05ab6_head_$rep.err || exit $?
  QOC_BLKP_TAIL=0 timeout -k 10 300 python bench.py --config tunable_bus --no-cpu > gpurun_out/r05ab6_eq_$rep.json 2> gpurun_out/r05ab6_eq_$rep.err || exit $?
  python -c "
import json
v=[json.load(open('gpurun_out/r05ab6_%s_$rep.json'%t)) for t in ('prev','head','eq')]
print('prev', round(v[0]['value'],1), ' head', round(v[1]['value'],1), ' head-equal-groups', round(v[2]['value'],1))"
done
