mkdir -p gpurun_out
export JLA_TUNE_FILE=$PWD/gpurun_out/tune_r4.json
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_suite.txt 2>&1
rc=$?
tail -3 gpurun_out/r4_gpu_suite.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --json-out gpurun_out/r4_bench2.json > gpurun_out/r4_bench2.log 2>&1 || exit $?
tail -2 gpurun_out/r4_bench2.log
