mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread -k "256x128" > gpurun_out/g4n_tests.txt 2>&1
rc=$?
tail -15 gpurun_out/g4n_tests.txt
[ $rc -ne 0 ] && exit $rc
B="timeout -k 10 300 python -u tools/bench_gemm.py"
$B --ops o down --mode residual --m 2048 1024 --tile 7 10 --ksplit 1 2 --rounds 2 --no-blas > gpurun_out/g4n.jsonl 2>&1 || exit $?
$B --ops gate_up --mode swiglu --rms --m 2048 1024 --tile 7 10 --rounds 2 --no-blas >> gpurun_out/g4n.jsonl 2>&1 || exit $?
$B --ops qkv lm_head --rms --m 2048 --tile 7 10 --rounds 2 --no-blas >> gpurun_out/g4n.jsonl 2>&1
grep '"us"' gpurun_out/g4n.jsonl
