mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/model_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/model_gpu.log; exit $rc
