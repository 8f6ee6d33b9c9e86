set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "packed or decode_linear_paths or tiled_splitk" > gpurun_out/t_pack.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 40 48 64 > gpurun_out/dp_pack32.log 2>&1
JLA_PACKED_X_MAX_M=64 timeout -k 10 300 python -u tools/decode_point.py --model llama3-8b --batch 40 48 64 --tune-report > gpurun_out/dp_pack64.log 2>&1
