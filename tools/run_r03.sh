#!/bin/bash
# Round-3 GPU check: focused tests (pytest -k expression $2, optional), the full -m gpu suite, the default bench
# and smoke; every step time-limited, the call ends at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03}
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests -k "$2" > gpurun_out/${T}_focus.log 2>&1 || exit 1
fi
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_cavity.json 2> gpurun_out/${T}_bench_cavity.err || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo done
