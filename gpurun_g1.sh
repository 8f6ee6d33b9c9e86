set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention_decode" > gpurun_out/t_attn.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_production_shapes_gpu.py > gpurun_out/t_model.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 40 48 64 > gpurun_out/dp_v4pack.log 2>&1
