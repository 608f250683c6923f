#!/bin/bash
# State-side gradient pass beside the first backward range (QOC_BWD_PRESTATE): parity test, then an
# alternating same-box A/B of the cavity and zz bench lines (each step time-limited).
set -o pipefail
o=gpurun_out/prestate
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k overlapped > $o/focus.log 2>&1 || exit 1
for rep in 1 2; do
  for cfg in cavity zz_batch; do
    for pre in 0 1; do
      QOC_BWD_PRESTATE=$pre timeout -k 10 120 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > $o/${cfg}_p${pre}_r${rep}.json 2> $o/${cfg}_p${pre}_r${rep}.err || exit 1
    done
  done
done
echo done
