#!/bin/bash
# fused greedy argmax: kernel test, model suites, then the default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "argmax" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_argmax.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1
