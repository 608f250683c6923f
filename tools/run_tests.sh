#!/bin/bash
# GPU test pass: the focused tests given as arguments (pytest -k expression, optional), then the full -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ -n "$1" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests -k "$1" > gpurun_out/${TAG}_focus.log 2>&1 || exit 1
fi
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gputest.log 2>&1 || exit 1
echo done
