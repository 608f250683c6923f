# GPU test suite + benches of every config (run on the GPU box from the repo root): tools/run_full.sh <tag>
T=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${T}_gputest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/${T}_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_cavity.json 2> gpurun_out/${T}_bench.err || exit 1
for c in zz_batch tunable_bus synthetic; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2>> gpurun_out/${T}_bench.err || exit 1
done
