#!/usr/bin/env bash
# Decode-only kernel breakdowns (tools/decode_breakdown.py) of one decode point per batch, e.g. the TP8 rank proxy:
#   bash tools/proxy_profile.sh gpurun_out/proxy "--model llama3-70b --tp-proxy 8" 1 32 256
# One rocprofv3 kernel-trace run per batch (prefill and autotune excluded by the breakdown), then
# <out>/b<B>.txt per batch. Stops at the first failing step.
set -euo pipefail
OUT=$1
ARGS=$2
shift 2
R=$(pwd)
mkdir -p "$R/$OUT"
for B in "$@"; do
  D="$R/$OUT/b$B"
  mkdir -p "$D"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$D" -o run -- \
    python3 "$R/tools/decode_point.py" $ARGS --batch "$B" --steps 32 > "$D/point.log" 2>&1)
  T=$(find "$D" -name run_kernel_trace.csv | head -n 1 || true)
  python3 tools/decode_breakdown.py "$T" --layers "${LAYERS:-80}" > "$R/$OUT/b$B.txt"
  tail -1 "$D/point.log" >> "$R/$OUT/b$B.txt"
  rm -f "$T"
  echo "batch $B done"; head -3 "$R/$OUT/b$B.txt"
done
