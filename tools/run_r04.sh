#!/bin/bash
# Round-4 GPU check: focused tests (pytest -k expression $2 over tests $3, optional), benches of the configs in $4
# (default "cavity zz_batch"), each step time-limited; the call ends at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04}
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${3:-tests} -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
for cfg in ${4:-cavity zz_batch}; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.err || exit 1
done
echo done
