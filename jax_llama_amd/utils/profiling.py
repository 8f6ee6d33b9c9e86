"""Tracing / profiling helpers (the reference has none: only ad-hoc prints, model.py:636-637,
generation.py:23-66).

* ``range(name)``: a roctx range (``torch.cuda.nvtx`` is roctx on ROCm) around a region so it
  shows up in ``rocprofv3 --marker-trace`` timelines; no-op on CPU.
* ``GpuTimer``: hipEvent-based device timer for a region (what bench.py's ms/step uses).
* ``kernel_summary(csv)``: per-kernel time table from a ``rocprofv3 --kernel-trace --stats``
  ``*_kernel_stats.csv`` (see tools/profile.sh).
* ``decode_breakdown(trace_csv)``: groups a kernel trace into the decode layer's stages.
"""
from __future__ import annotations

import contextlib
import csv
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class GpuTimer:
    """``with GpuTimer() as t: ...; t.ms`` -- device time between two hipEvents (host wall time
    on CPU)."""

    def __init__(self, sync: bool = True):
        self.sync = sync
        self.ms: Optional[float] = None

    def __enter__(self):
        if torch.cuda.is_available():
            self._a = torch.cuda.Event(enable_timing=True)
            self._b = torch.cuda.Event(enable_timing=True)
            self._a.record()
        else:
            self._t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if torch.cuda.is_available():
            self._b.record()
            if self.sync:
                self._b.synchronize()
                self.ms = self._a.elapsed_time(self._b)
        else:
            self.ms = 1000.0 * (time.perf_counter() - self._t)
        return False


def kernel_summary(stats_csv: str, top: int = 25) -> List[Dict]:
    """Rows of a rocprofv3 ``kernel_stats.csv`` sorted by total time."""
    rows = list(csv.DictReader(open(stats_csv)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    out = []
    for r in rows[:top]:
        out.append({"kernel": r["Name"][:100], "calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                    "avg_us": float(r["AverageNs"]) / 1e3, "pct": float(r["Percentage"])})
    return out


_STAGES = (("linear_skinny_kernel", "decode GEMV"), ("skinny_kernel", "decode split-K GEMM"),
           ("gemm_kernel", "prefill GEMM"), ("attn_decode", "decode attention"),
           ("attn_prefill", "prefill attention"), ("rope_kv", "rope+kv write"), ("rms_kernel", "rmsnorm"),
           ("embedding", "embedding"), ("argmax", "sampler"), ("decode_update", "sampler"),
           ("topk", "sampler"))


def decode_breakdown(trace_csv: str) -> Dict[str, float]:
    """Total device ms per stage from a rocprofv3 ``kernel_trace.csv``."""
    tot: Dict[str, float] = defaultdict(float)
    for r in csv.DictReader(open(trace_csv)):
        name = r.get("Kernel_Name", "")
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        stage = next((s for key, s in _STAGES if key in name), "other")
        tot[stage] += dur
    return dict(sorted(tot.items(), key=lambda kv: -kv[1]))
