set -o pipefail
mkdir -p gpurun_out/bb
for B in 4096 2048; do
timeout -k 10 500 python3 bench.py --batch $B --steps 2 --warmup 1 --latency-batches --no-sampled --ttft-len 0 --proxy-model '' --mp1-model '' --no-calibration --json-out gpurun_out/bb/b$B.json > gpurun_out/bb/b$B.log 2>&1 || { tail -20 gpurun_out/bb/b$B.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bb/b$B.json')); print($B, d['value'], d['ttft_ms'], d['decode_ms_per_token'], d['gemm_plan_choice'])"
done
