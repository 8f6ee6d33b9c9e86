set -o pipefail
mkdir -p gpurun_out
for sh in 8b_b16_s2048 7b_b16_s2048 8b_b1_s8192; do
  timeout -k 10 200 python -u tools/bench_attn_prefill.py --shape $sh --impls 13 7 --rounds 6 >> gpurun_out/pf_disp.jsonl 2>&1 || exit $?
done
grep shape gpurun_out/pf_disp.jsonl
