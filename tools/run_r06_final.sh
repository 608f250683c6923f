#!/bin/bash
# round-6 final check: the GPU test suite, smoke(), the default bench line (with its side legs), then every config's
# bench lines (tools/run_r06_bench.sh).  Usage: <tag>
set -o pipefail
T=${1:-r06h}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_gputest.log 2>&1 || { tail -30 gpurun_out/${T}_gputest.log; exit 1; }
tail -2 gpurun_out/${T}_gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${T}_default.json 2> gpurun_out/${T}_default.err || exit 1
timeout -k 10 1000 tools/run_r06_bench.sh $T || exit 1
echo final done
