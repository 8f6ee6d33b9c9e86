mkdir -p gpurun_out
export JLA_TUNE_FILE=$PWD/gpurun_out/tune_r4.json
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_tp_proxy_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r4_tp_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r4_tp_tests.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 1000 python -u bench.py --steps 2 --warmup 1 --json-out gpurun_out/r4_bench3.json > gpurun_out/r4_bench3.log 2>&1 || exit $?
tail -1 gpurun_out/r4_bench3.log | cut -c1-300
