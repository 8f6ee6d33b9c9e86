mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread -k "chained or every_epilogue" > gpurun_out/g4_chain_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/g4_chain_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm.py --ops o down --mode residual --m 2048 1024 --tile 7 9 --ksplit 1 2 --rounds 1 --no-blas > gpurun_out/g4_chain.jsonl 2>&1
rc=$?
grep '"us"' gpurun_out/g4_chain.jsonl
exit $rc
