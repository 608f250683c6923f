#!/bin/bash
# Occupancy probe: evals/s against seeds per GPU (more resident waves) + kernel traces of zz and tunable bus.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for s in 256 1024 2048; do
  timeout -k 10 300 python bench.py --config zz_batch --seeds $s --no-cpu --steps 20 > gpurun_out/r03g_zz_$s.json 2>/dev/null || exit 1
done
for s in 128 512; do
  timeout -k 10 300 python bench.py --config cavity --seeds $s --no-cpu --steps 10 > gpurun_out/r03g_cav_$s.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --config tunable_bus --seeds 1024 --no-cpu --steps 5 > gpurun_out/r03g_tb_1024.json 2>/dev/null || exit 1
for c in zz_batch tunable_bus; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03g_trace_$c -o run -- python bench.py --config $c --no-cpu --steps 5 --warmup 2 > gpurun_out/r03g_trace_$c.log 2>&1 || exit 1
done
echo done
