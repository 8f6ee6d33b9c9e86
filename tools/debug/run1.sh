set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -5 | tee gpurun_out/g4_tests3.log
B="timeout -k 10 300 python -u tools/bench_gemm.py"
$B --ops gate_up qkv o down lm_head --m 2048 1024 --tile 7 8 --rounds 2 --no-blas | tee gpurun_out/g4_sk.jsonl
$B --ops gate_up --mode swiglu --rms --m 2048 --tile 7 8 --rounds 2 --no-blas | tee -a gpurun_out/g4_sk.jsonl
$B --ops o down --mode residual --m 2048 --tile 7 8 --ksplit 1 2 --rounds 2 --no-blas | tee -a gpurun_out/g4_sk.jsonl
