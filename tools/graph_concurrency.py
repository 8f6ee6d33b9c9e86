#!/usr/bin/env python3
"""Do two captured streams of a hipGraph run concurrently on this ROCm? (the premise of overlapping decode attention
of one micro-batch with another's GEMMs, and of side-stream weight prefetch).

A deliberately narrow streaming kernel (ops.prefetch over 1 GiB with 16 workgroups: bandwidth-light, latency-long) is
run once (A), twice in sequence on one stream (AA), and once on each of two streams forked / joined inside one graph
(A||A); the same three eagerly. Concurrent branches give A||A ~= A, serialized ones ~= AA.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402


def main():
    e = ops.ext()
    a = torch.empty(1 << 28, dtype=torch.int32, device="cuda")  # 1 GiB
    b = torch.empty(1 << 28, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    e.prefetch(a, 16)  # first call allocates the sink (never under capture)
    torch.cuda.synchronize()

    def one():
        e.prefetch(a, 16)

    def seq():
        e.prefetch(a, 16)
        e.prefetch(b, 16)

    def par():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        e.prefetch(a, 16)
        with torch.cuda.stream(side):
            e.prefetch(b, 16)
        main.wait_stream(side)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    for name, fn in (("A", one), ("AA", seq), ("A||A", par)):
        fn()
        torch.cuda.synchronize()
        ev0.record()
        fn()
        ev1.record()
        ev1.synchronize()
        out["eager_" + name] = round(ev0.elapsed_time(ev1), 3)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        ev0.record()
        g.replay()
        ev1.record()
        ev1.synchronize()
        out["graph_" + name] = round(ev0.elapsed_time(ev1), 3)
    out["unit"] = "ms"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
