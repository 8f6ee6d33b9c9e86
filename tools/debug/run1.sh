set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py tests/test_production_shapes_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -5 | tee gpurun_out/r4_tests_a.log
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --json-out gpurun_out/r4_bench_g4.json 2>&1 | tail -3
