set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention_decode" > gpurun_out/t_attn.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 128 256 > gpurun_out/dp_8b_mid.log 2>&1
timeout -k 10 400 python -u tools/decode_point.py --model llama3-70b --batch 256 > gpurun_out/dp_70b_b256.log 2>&1
