# Kernel sequence of one captured decode step (B = 1, Llama-3-8B): rocprofv3 kernel trace of tools/decode_point.py,
# then the last step's dispatches in order with their durations
set -o pipefail
OUT=${1:-gpurun_out/step_seq}
R=$(pwd)
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT" -o run -- \
  python3 "$R/tools/decode_point.py" --batch 1 --steps 8 > "$R/$OUT/dp.log" 2>&1 || { echo "rocprof rc=$?"; tail -20 "$R/$OUT/dp.log"; exit 1; }
cd "$R"
T=$(ls $OUT/run_kernel_trace.csv $OUT/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$T" > "$OUT/seq.txt" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in csv.DictReader(open(sys.argv[1])))
emb = [i for i, r in enumerate(rows) if "embedding_kernel" in r[2]]
a, b = emb[-2], emb[-1]
for s, e, n in rows[a:b]:
    print(f"{(e - s) / 1000:8.2f} us  {n.replace('void ', '').replace('jla::', '')[:80]}")
print("step wall", (rows[b][0] - rows[a][0]) / 1000, "us")
PY
cat "$OUT/seq.txt"
rm -f "$T"
