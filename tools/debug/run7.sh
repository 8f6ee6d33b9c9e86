set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention_prefill_long" -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -3 gpurun_out/pf_tests.log
timeout -k 10 400 python -u tools/bench_attn_prefill.py --impls 2 9 13 7 --rounds 3 > gpurun_out/pf_ab.jsonl 2>&1
cat gpurun_out/pf_ab.jsonl
