#!/usr/bin/env python3
"""Group a rocprofv3 kernel trace by (kernel, grid, workgroup) -> calls / total / avg.

Decode-step launches of one shape repeat every step, so grouping by launch geometry separates the
prefill GEMMs from the decode GEMMs of the same kernel template (and the shapes from each other).

  python tools/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--top 40] [--json out.json]
  python tools/trace_breakdown.py gpurun_out/prof/run_results.db     (rocprofv3's default rocpd output)
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)           # drop the argument list
    name = name.replace("void ", "").replace("jla::", "")
    return name[:60]


def _records(path: str):
    """(name, grid, workgroup, duration_us) per dispatch, from a kernel-trace CSV or a rocpd SQLite db."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        for name, gx, gy, gz, wx, wy, wz, dur in con.execute(
                "select name, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, duration from kernels"):
            yield name, str(gx * gy * gz), str(wx * wy * wz), dur / 1e3
        return
    for r in csv.DictReader(open(path)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        wg = r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?"))
        yield r.get("Kernel_Name", "?"), grid, wg, dur


def breakdown(path: str):
    groups = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for name, grid, wg, dur in _records(path):
        key = (short(name), grid, wg)
        g = groups[key]
        g[0] += 1
        g[1] += dur
        total += dur
    rows = [{"kernel": k[0], "grid": k[1], "wg": k[2], "calls": v[0], "total_ms": round(v[1] / 1e3, 3),
             "avg_us": round(v[1] / v[0], 2), "pct": round(100 * v[1] / total, 2)} for k, v in groups.items()]
    rows.sort(key=lambda r: -r["total_ms"])
    return rows, total / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows, total = breakdown(a.trace)
    print(f"total kernel time {total:.1f} ms")
    print(f"{'kernel':60s} {'grid':>9s} {'wg':>4s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>6s}")
    for r in rows[: a.top]:
        print(f"{r['kernel']:60s} {r['grid']:>9s} {r['wg']:>4s} {r['calls']:6d} {r['total_ms']:9.2f} "
              f"{r['avg_us']:9.2f} {r['pct']:6.2f}")
    if a.json:
        json.dump({"total_ms": total, "groups": rows}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
