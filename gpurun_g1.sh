set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tp_proxy_gpu.py tests/test_car_failure_gpu.py "tests/test_tp_gpu.py::test_tp_decode_matches_single_process[2-small-4]" "tests/test_tp_gpu.py::test_tp_decode_matches_single_process[2-small-12]" > gpurun_out/t_fused.log 2>&1
timeout -k 10 240 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 1 32 > gpurun_out/dp_fused.log 2>&1
JLA_TP_FUSED=0 timeout -k 10 240 python -u tools/decode_point.py --model llama3-70b --tp-proxy 8 --batch 1 32 > gpurun_out/dp_unfused.log 2>&1
