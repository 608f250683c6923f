timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_gputest.log 2>&1
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/$1_bench_cav.json 2> gpurun_out/$1_bench.err
timeout -k 10 200 python bench.py --no-cpu --config zz_batch > gpurun_out/$1_bench_zz.json 2>> gpurun_out/$1_bench.err
