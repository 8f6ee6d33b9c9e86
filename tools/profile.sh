#!/usr/bin/env bash
# Kernel-level profile of the headline benchmark on one MI355X (run via gpurun from the repo root):
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/profile.sh gpurun_out/prof'
# Writes <out>/run_kernel_stats.csv (+ trace) and a JSON stage breakdown. Counters (--pmc) are
# collected in a separate run (never combined with tracing domains other than kernel-trace).
set -euo pipefail
OUT=${1:-gpurun_out/prof}
shift || true
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --gen-len 64 "$@" > "$R/$OUT/bench.log" 2>&1
cd "$R"
python3 - "$OUT" <<'EOF'
import json, sys
sys.path.insert(0, ".")
from jax_llama_amd.utils.profiling import decode_breakdown, kernel_summary
out = sys.argv[1]
summary = {"kernels": kernel_summary(f"{out}/run_kernel_stats.csv"),
           "stages_ms": decode_breakdown(f"{out}/run_kernel_trace.csv")}
json.dump(summary, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summary["stages_ms"], indent=1))
EOF
