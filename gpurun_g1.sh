set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "qkv" tests/test_model_gpu.py tests/test_production_shapes_gpu.py > gpurun_out/t_qkvd.log 2>&1
JLA_QKV_DIRECT=0 timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 2048 --steps 16 > gpurun_out/qkvd0.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 2048 --steps 16 > gpurun_out/qkvd1.log 2>&1
JLA_QKV_DIRECT=0 timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 2048 --steps 16 > gpurun_out/qkvd0b.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 2048 --steps 16 > gpurun_out/qkvd1b.log 2>&1
