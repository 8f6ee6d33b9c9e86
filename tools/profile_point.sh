#!/usr/bin/env bash
# Kernel trace of one decode latency point (tools/decode_point.py), e.g. the one-GPU TP rank proxy:
#   bash tools/profile_point.sh gpurun_out/prof_proxy --model llama3-70b --tp-proxy 8 --batch 1 --steps 32
# Writes <out>/run_kernel_trace.csv + run_kernel_stats.csv and <out>/breakdown.txt (tools/trace_breakdown.py).
set -euo pipefail
OUT=${1:-gpurun_out/prof_point}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT" -o run -- \
  python3 "$R/tools/decode_point.py" "$@" > "$R/$OUT/point.log" 2>&1
cd "$R"
python3 tools/trace_breakdown.py "$OUT/run_kernel_trace.csv" --top 40 > "$OUT/breakdown.txt"
