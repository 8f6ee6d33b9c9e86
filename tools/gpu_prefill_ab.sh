# A/B of the software-pipelined flash prefill (impl 7 / 9) and lazy rescale (impl 8) against the defaults,
# after the prefill numerics tests for every impl (fp32 reference)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill" > gpurun_out/pf_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -2 gpurun_out/pf_tests.log
timeout -k 10 300 python -u tools/bench_attn_prefill.py --impls 2 7 8 5 9 --rounds 4 > gpurun_out/pf_ab.jsonl 2>&1 || { echo ab rc=$?; tail -20 gpurun_out/pf_ab.jsonl; exit 1; }
cat gpurun_out/pf_ab.jsonl
timeout -k 10 300 python -u tools/bench_attn_decode.py --shapes 2048x128 2048x256 2048x384 256x384 --impls 2 12 --rounds 4 > gpurun_out/v4_lazy_ab.jsonl 2>&1 || { echo v4ab rc=$?; tail -20 gpurun_out/v4_lazy_ab.jsonl; exit 1; }
cat gpurun_out/v4_lazy_ab.jsonl
