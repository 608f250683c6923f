#!/bin/bash
# full GPU suite after the stored-propagator path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g_gputest.log 2>&1
rc=$?; tail -5 gpurun_out/r05g_gputest.log; exit $rc
