set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_allreduce_gpu.py tests/test_car_failure_gpu.py tests/test_tp_proxy_gpu.py > gpurun_out/t_car.log 2>&1
JLA_CAR_GRID=63 timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 256 > gpurun_out/dp_grid63.log 2>&1
timeout -k 10 300 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 256 32 1 > gpurun_out/dp_grid255.log 2>&1
