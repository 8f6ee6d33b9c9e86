mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_decode_mk_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mk_tests.txt 2>&1
rc=$?
tail -30 gpurun_out/mk_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/bench_decode_mk.py --batches 1 4 --rounds 2 > gpurun_out/mk_bench.jsonl 2>&1
rc=$?
cat gpurun_out/mk_bench.jsonl | grep decode_ms
exit $rc
