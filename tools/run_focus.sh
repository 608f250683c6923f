#!/bin/bash
# focused GPU tests (tools/run_focus.sh <tag> <pytest paths or -k expr...>) into gpurun_out/<tag>_focus.log
set -o pipefail
T=${1:-r06}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/${T}_focus.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_focus.log; exit $rc
