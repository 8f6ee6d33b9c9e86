set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention_decode" > gpurun_out/t_attn.log 2>&1
timeout -k 10 300 python -u tools/bench_kernels.py --ops attn --attn-impls 2:4096,102:4096 --attn-shapes 2048x128 2048x256 2048x384 1024x384 > gpurun_out/attn_v4fast.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 2048 --steps 16 > gpurun_out/dp2048_v4fast.log 2>&1
