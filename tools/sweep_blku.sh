#!/bin/bash
# Block-propagator shape sweep: formation waves (QOC_BLKU_FW) x slices per chunk (QOC_BLKU_C) per config; one bench
# line each (no CPU baseline), summary in gpurun_out/$1_sweep.txt.  Each run time-limited; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04s}
out=gpurun_out/${T}_sweep.txt
: > $out
for cfg in ${2:-cavity zz_batch}; do
  for fw in ${3:-1 2 3 4}; do
    for c in ${4:-16 32}; do
      QOC_BLKU_FW=$fw QOC_BLKU_C=$c timeout -k 10 120 python bench.py --config $cfg --no-cpu --steps 10 > gpurun_out/${T}_${cfg}_fw${fw}_c${c}.json 2>/dev/null || exit 1
      python - "$cfg" "$fw" "$c" gpurun_out/${T}_${cfg}_fw${fw}_c${c}.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[1], "fw", sys.argv[2], "C", sys.argv[3], "evals/s %.0f" % d["value"], "step %.4f" % d["ms_per_step"],
      "chain %.4f" % k["k_chain_fwd"]["ms_per_launch"], "grad %.4f" % k["k_grad"]["ms_per_launch"])
PY
    done
  done
done
cat $out
