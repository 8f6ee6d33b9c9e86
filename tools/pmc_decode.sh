#!/usr/bin/env bash
# PMC counters of one decode point (tools/decode_point.py), two passes (the per-block counter limits): SQ cycles /
# MFMA busy, then HBM fetch bytes. Usage (repo root, via gpurun):
#   bash tools/pmc_decode.sh gpurun_out/pmc_b2048 --model llama3-8b --batch 2048 --steps 4
# Writes <out>/sq/... and <out>/mem/... (rocprofv3 csv) and <out>/summary_{sq,mem}.txt (tools/pmc_summary.py).
set -euo pipefail
OUT=${1:-gpurun_out/pmc_decode}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT/sq" "$R/$OUT/mem"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$R/$OUT/sq" -o run -- python3 "$R/tools/decode_point.py" "$@" > "$R/$OUT/sq/log.txt" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/$OUT/mem" -o run -- python3 "$R/tools/decode_point.py" "$@" > "$R/$OUT/mem/log.txt" 2>&1
cd "$R"
python3 tools/pmc_summary.py "$OUT/sq/run_counter_collection.csv" > "$OUT/summary_sq.txt"
python3 tools/pmc_summary.py "$OUT/mem/run_counter_collection.csv" > "$OUT/summary_mem.txt"
