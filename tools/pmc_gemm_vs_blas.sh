#!/usr/bin/env bash
# PMC counters of gemm2 and hipBLASLt on the same shapes (two passes: SQ block, then TA/TCP/GRBM).
# Usage (repo root, via gpurun): bash tools/pmc_gemm_vs_blas.sh <outdir> [bench_gemm args...]
set -euo pipefail
OUT=${1:-gpurun_out/pmcb}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$R/$OUT/sq" -o run -- python3 "$R/tools/bench_gemm.py" "$@" > "$R/$OUT/log_sq.txt" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum \
  TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$R/$OUT/ta" -o run -- python3 "$R/tools/bench_gemm.py" "$@" > "$R/$OUT/log_ta.txt" 2>&1
cd "$R"
for p in sq ta; do
  f=$(ls $OUT/$p/run_counter_collection.csv 2>/dev/null || true)
  [ -n "$f" ] && python3 tools/pmc_summary.py "$f" > "$OUT/summary_$p.txt"
done
