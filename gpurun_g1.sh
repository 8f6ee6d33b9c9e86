set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "split_gemv or decode_linear_paths or packed_x_variants or qkv_rope_fused or variants_agree" > gpurun_out/t_split.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_tp_proxy_gpu.py > gpurun_out/t_proxy.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 1 32 > gpurun_out/dp_proxy.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 1 32 64 > gpurun_out/dp_8b.log 2>&1
