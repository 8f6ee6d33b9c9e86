set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention_decode" > gpurun_out/t_attn.log 2>&1
timeout -k 10 300 python -u tools/bench_attn_decode.py --model llama3-70b --tp 8 --shapes 1x192 1x384 8x384 32x384 --cache-len 384 --impls 6 5 > gpurun_out/attn_fold_70b.log 2>&1
timeout -k 10 300 python -u tools/bench_attn_decode.py --model llama3-8b --shapes 1x192 1x384 8x384 16x384 --cache-len 384 --impls 6 5 > gpurun_out/attn_fold_8b.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 1 32 > gpurun_out/dp_proxy.log 2>&1
