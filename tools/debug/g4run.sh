# gemm4 bring-up on one GPU: numerics tests, then library A/B vs gemm2 and hipBLASLt
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm4_gpu.py -x -v --timeout 120 --timeout-method thread -s 2>&1 | tee gpurun_out/g4_tests.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 2048 4096 32768 --tile 1 7 --rounds 2 | tee gpurun_out/g4_bench2.jsonl
