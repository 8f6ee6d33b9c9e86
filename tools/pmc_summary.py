#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per (kernel, grid) from a counter_collection.csv."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
acc = defaultdict(lambda: defaultdict(list))
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:50]
    key = (name, r.get("Grid_Size", "?"))
    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in acc.items():
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    line = f"{key[0]:50s} grid={key[1]:>9s} n={len(next(iter(cs.values())))}"
    for k in sorted(avg):
        line += f" {k}={avg[k]:.4g}"
    if "SQ_BUSY_CYCLES" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        line += f" | mfma_busy/busy={avg['SQ_VALU_MFMA_BUSY_CYCLES'] / max(avg['SQ_BUSY_CYCLES'], 1):.3f}"
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in avg:
            line += f" {k[3:]}/wave={avg[k] / wc:.3f}"
    print(line)
