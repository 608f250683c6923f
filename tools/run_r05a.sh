#!/bin/bash
# round 5: first GPU check of the segmented block eval (tests + short benches)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_blkseg.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r05a_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config cavity --steps 20 --warmup 3 --no-cpu > gpurun_out/r05a_bench_cavity.json 2> gpurun_out/r05a_bench_cavity.err || exit $?
timeout -k 10 300 python bench.py --config zz_batch --steps 20 --warmup 3 --no-cpu > gpurun_out/r05a_bench_zz.json 2> gpurun_out/r05a_bench_zz.err || exit $?
python - <<'PY'
import json
for n in ("cavity", "zz"):
    d = json.load(open(f"gpurun_out/r05a_bench_{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["engine"]["backward"])
PY
