set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "prefill or attention or ttft or generate" -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_tests2.log 2>&1 || { tail -30 gpurun_out/pf_tests2.log; exit 1; }
tail -2 gpurun_out/pf_tests2.log
timeout -k 10 300 python -u tools/ttft.py --prompt-len 2048 8192 > gpurun_out/ttft.log 2>&1; tail -5 gpurun_out/ttft.log
