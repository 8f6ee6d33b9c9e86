set -o pipefail
OUT=gpurun_out/prof8
R=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 1 --gen-len 64 --latency-batches --no-sampled --ttft-len 0 --proxy-model '' --mp1-model '' --no-calibration > "$R/$OUT/bench.log" 2>&1 || { echo rc=$?; tail -20 "$R/$OUT/bench.log"; exit 1; }
cd "$R"
T=$(ls $OUT/run_kernel_trace.csv $OUT/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_breakdown.py "$T" --top 45 > $OUT/breakdown.txt
rm -f "$T"
cat $OUT/breakdown.txt
tail -2 $OUT/bench.log
