set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm4_gpu.py tests/test_kernels_gpu.py -k "gemm4 or qkv or residual or reduce or attention_prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/g4_tests.log 2>&1 || { tail -30 gpurun_out/g4_tests.log; exit 1; }
tail -2 gpurun_out/g4_tests.log
B="timeout -k 10 300 python -u tools/bench_gemm.py"
$B --ops o down --mode residual --m 32768 2048 --tile 7 --ksplit 1 2 --rounds 2 --no-blas > gpurun_out/g_resid.jsonl 2>&1
grep -h '"op"' gpurun_out/g_resid.jsonl
