#!/usr/bin/env bash
# Memory-side PMC counters (TA / TCP / TCC) of the tiled GEMM; companion of tools/pmc_gemm.sh.
set -euo pipefail
OUT=${1:-gpurun_out/pmc_mem}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum \
  TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/$OUT" -o run -- python3 "$R/tools/bench_gemm.py" --no-blas "$@" > "$R/$OUT/log.txt" 2>&1
