# impl 11 / 12 (branch-free pipelined body) vs 7 / 9 and the default: numerics against the fp32 reference first
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "
import torch, sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import test_kernels_gpu as t
for impl in (11, 12):
    for rep in (1, 4, 8):
        for s, slot0, masked in ((7, 0, False), (130, 10, False), (512, 0, False), (300, 0, True), (2048, 0, False)):
            t.test_attention_prefill_long(impl, rep, s, slot0, masked)
print('impl 11/12 numerics ok')
" > gpurun_out/pipe2_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pipe2_tests.log; exit 1; }
tail -1 gpurun_out/pipe2_tests.log
timeout -k 10 300 python -u tools/bench_attn_prefill.py --impls 2 11 12 7 9 --rounds 4 > gpurun_out/pf_ab2.jsonl 2>&1 || { echo ab rc=$?; tail -20 gpurun_out/pf_ab2.jsonl; exit 1; }
cat gpurun_out/pf_ab2.jsonl
