# A/B of the flash prefill default (impl 2: lazy rescale + software pipelining) against the previous default (10)
# and the explicit pipelined 4 / 8-wave launches (7 / 9),
# after the prefill numerics tests for every impl (fp32 reference)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill" > gpurun_out/pf_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -2 gpurun_out/pf_tests.log
timeout -k 10 300 python -u tools/bench_attn_prefill.py --impls 2 10 7 9 --rounds 4 > gpurun_out/pf_ab.jsonl 2>&1 || { echo ab rc=$?; tail -20 gpurun_out/pf_ab.jsonl; exit 1; }
cat gpurun_out/pf_ab.jsonl
timeout -k 10 300 python -u tools/ttft.py --prompt-len 2048 8192 > gpurun_out/pf_ttft.jsonl 2>&1 || { echo ttft rc=$?; tail -20 gpurun_out/pf_ttft.jsonl; exit 1; }
cat gpurun_out/pf_ttft.jsonl
