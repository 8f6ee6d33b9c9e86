set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/profile_point.sh gpurun_out/prof_proxy_b1 --model llama3-70b --tp-proxy 8 --batch 1 --steps 32
bash tools/profile_point.sh gpurun_out/prof_8b_b1 --model llama3-8b --batch 1 --steps 32
timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
