#!/bin/bash
# Probe runs of the block-propagator kernels ($1: tag): the focused block tests ($2 over $3), the segment breakdown
# of k_blku_fwd / k_blku_bwdg (tools/blku_probe) on the cavity (NB=2) and zz (NB=3) shapes, then benches of cavity
# and zz; each step time-limited, stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04p}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${3:-tests} -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
timeout -k 10 300 tools/blku_probe 2 > gpurun_out/${T}_probe2.txt 2>&1 || exit 1
timeout -k 10 200 tools/blku_probe 3 > gpurun_out/${T}_probe3.txt 2>&1 || exit 1
for cfg in cavity zz_batch; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.err || exit 1
done
echo done
