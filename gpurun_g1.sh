set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "packed_x_variants" > gpurun_out/t_v23.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 64 32 16 --tune-report > gpurun_out/tune_v23.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 32 --tune-report > gpurun_out/tune_v23p.log 2>&1
