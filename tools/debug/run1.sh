set -e
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tee gpurun_out/r4_gpu_suite.log | tail -15
