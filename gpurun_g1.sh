set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/pmc_decode.sh gpurun_out/pmc_b2048 --model llama3-8b --batch 2048 --steps 4
