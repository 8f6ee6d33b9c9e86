set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_attn_prefill.py --impls 2 4 5 6 --rounds 4 > gpurun_out/prefill_nw8b.log 2>&1
