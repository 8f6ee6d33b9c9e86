set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "skinny_argmax or decode_linear_paths or packed_x_variants" > gpurun_out/t_v20.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 1 32 --tune-report > gpurun_out/tune_proxy2.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 1 32 --tune-report > gpurun_out/tune_8b2.log 2>&1
