#!/usr/bin/env bash
# SQ counters of the decode attention kernels at one shape (tools/bench_attn_decode.py; graph replays), e.g.
#   bash tools/pmc_attn.sh gpurun_out/pmc_attn --model llama3-70b --shapes 256x256 --impls 2 62
set -euo pipefail
OUT=${1:-gpurun_out/pmc_attn}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT/sq"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/$OUT/sq" -o run -- python3 "$R/tools/bench_attn_decode.py" --reps 4 --rounds 1 "$@" \
  > "$R/$OUT/sq/log.txt" 2>&1
cd "$R"
python3 tools/pmc_summary.py "$OUT/sq/run_counter_collection.csv" > "$OUT/summary_sq.txt"
cat "$OUT/summary_sq.txt"
