#!/usr/bin/env python3
"""Decode-only per-kernel breakdown of a ``tools/decode_point.py`` rocprofv3 kernel trace (one batch point per run).

``decode_latency`` runs: cold prefill, warm prefill, one eager step, graph capture + one replay, a third prefill,
then the timed replays. Everything after the LAST prefill-only dispatch (``--marker``, default the flash-prefill
kernel) is the timed replays, so prefill and autotune never enter the numbers. Per-step microseconds per
(kernel, grid) and a category split: gemm (GEMV / GEMM / split-K reduce), attention, allreduce (standalone custom
all-reduce launches; the GEMV-fused row-parallel exchange is inside its GEMV), sampler, other.

  python tools/decode_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict

CATS = (("attention", ("attn_decode",)),
        ("allreduce", ("car_", "allreduce")),
        ("sampler", ("argmax", "topk", "decode_update", "sample")),
        ("gemm", ("gemm", "gemv", "linear_", "reduce")),
        ("norm/embed/rope", ("rms", "embed", "rope", "norm")))


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("jla::", "")
    return name[:70]


def category(name: str) -> str:
    for cat, keys in CATS:
        if any(k in name for k in keys):
            return cat
    return "other"


def load(path: str):
    rows = []
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        rows.append((s, e, r.get("Kernel_Name", "?"), grid))
    rows.sort()
    return rows


def decode_rows(rows, marker: str, step_marker: str):
    last = max((i for i, r in enumerate(rows) if marker in r[2]), default=-1)
    # the first step starts at the first step-marker launch after the last prefill (drops the prefill's tail)
    first = next((i for i in range(last + 1, len(rows)) if step_marker in rows[i][2]), last + 1)
    tail = rows[first:]
    steps = sum(1 for r in tail if step_marker in r[2])
    return tail, max(1, steps)


def breakdown(rows, steps):
    groups = defaultdict(lambda: [0, 0.0])
    cats = defaultdict(float)
    for s, e, name, grid in rows:
        us = (e - s) / 1e3
        k = (short(name), grid)
        groups[k][0] += 1
        groups[k][1] += us
        cats[category(short(name))] += us
    out = [{"kernel": k[0], "grid": k[1], "per_step": round(v[0] / steps, 2), "us_per_step": round(v[1] / steps, 2),
            "avg_us": round(v[1] / v[0], 2)} for k, v in groups.items()]
    out.sort(key=lambda r: -r["us_per_step"])
    wall = (rows[-1][1] - rows[0][0]) / 1e3 / steps if rows else 0.0
    return out, {c: round(t / steps, 1) for c, t in cats.items()}, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="attn_prefill")
    ap.add_argument("--step-marker", default="embedding")
    ap.add_argument("--layers", type=int, default=None, help="also print per-layer microseconds")
    ap.add_argument("--json", default=None)
    ap.add_argument("--sequence", type=int, default=12, help="print the first N launches of the last step in order")
    a = ap.parse_args()
    rows, steps = decode_rows(load(a.trace), a.marker, a.step_marker)
    groups, cats, wall = breakdown(rows, steps)
    ksum = sum(cats.values())
    print(f"decode steps {steps}; kernel time {ksum:.1f} us/step; wall (first start -> last end) {wall:.1f} us/step; "
          f"gaps {wall - ksum:.1f} us/step")
    print("by category (us/step): " + ", ".join(f"{c} {t}" for c, t in sorted(cats.items(), key=lambda x: -x[1])))
    if a.layers:
        print("by category (us/layer): " + ", ".join(f"{c} {round(t / a.layers, 2)}"
                                                     for c, t in sorted(cats.items(), key=lambda x: -x[1])))
    print(f"{'kernel':70s} {'grid':>9s} {'n/step':>7s} {'us/step':>9s} {'avg_us':>8s}")
    for g in groups:
        print(f"{g['kernel']:70s} {g['grid']:>9s} {g['per_step']:7.2f} {g['us_per_step']:9.2f} {g['avg_us']:8.2f}")
    if a.sequence:
        last = max(i for i, r in enumerate(rows) if a.step_marker in r[2])
        print(f"first {a.sequence} launches of the last step (us, gap to the previous end):")
        for j in range(last, min(len(rows), last + a.sequence)):
            s, e, name, grid = rows[j]
            gap = (s - rows[j - 1][1]) / 1e3 if j > 0 else 0.0
            print(f"  {(e - s) / 1e3:8.2f} {gap:6.2f}  {short(name)} grid {grid}")
    if a.json:
        json.dump({"steps": steps, "wall_us_per_step": wall, "kernel_us_per_step": ksum, "categories": cats,
                   "groups": groups}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
