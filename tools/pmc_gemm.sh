#!/usr/bin/env bash
# PMC counters of the tiled GEMM on one shape set (run from the repo root via gpurun).
# Usage: bash tools/pmc_gemm.sh <outdir> [bench_gemm args...]
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$R/$OUT" -o run -- python3 "$R/tools/bench_gemm.py" --no-blas "$@" > "$R/$OUT/log.txt" 2>&1
