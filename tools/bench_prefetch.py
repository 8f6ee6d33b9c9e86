#!/usr/bin/env python3
"""Does a decode GEMV read faster when its weights were just streamed into the Infinity Cache?

For each projection shape: hipGraph-replayed R x [fill 512 MiB (evicts the caches), (prefetch W), GEMV(W)], timed
as a difference against the same graph without the GEMV, so the number is the GEMV's own time (plus one kernel
boundary), cold vs after ops.prefetch. Prints one JSON line per (shape, mode).

  python tools/bench_prefetch.py --model llama3-70b --tp 8 --m 1
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402
from jax_llama_amd.config import get_preset  # noqa: E402
from jax_llama_amd.models.weights import PackedLinear  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    cfg = get_preset(args.model)
    d, f, hd = cfg.hidden_size, cfg.intermediate_size // args.tp, cfg.head_dim
    h, hkv = cfg.num_attention_heads // args.tp, cfg.num_key_value_heads // args.tp
    shapes = {"qkv": ((h + 2 * hkv) * hd, d), "o": (d, h * hd), "gate_up": (2 * f, d), "down": (d, f)}
    flush = torch.empty(512 << 18, dtype=torch.int32, device="cuda")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, (n, k) in shapes.items():
        w = PackedLinear.random(n, k, "cuda", 0.02, torch.Generator(device="cuda").manual_seed(1))
        x = torch.randn(args.m, k, device="cuda").to(torch.bfloat16)
        ops.linear(x, w)  # autotune outside capture
        ops.prefetch(w.weight)  # (first call allocates the sink)
        torch.cuda.synchronize()
        graphs = {}
        for mode in ("cold", "prefetched"):
            for with_gemv in (True, False):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(args.reps):
                        flush.fill_(1)
                        if mode == "prefetched":
                            ops.prefetch(w.weight)
                        if with_gemv:
                            ops.linear(x, w)
                graphs[(mode, with_gemv)] = g
        best = {"cold": float("inf"), "prefetched": float("inf")}
        for _ in range(args.rounds):
            for mode in best:
                t = {}
                for with_gemv in (True, False):
                    g = graphs[(mode, with_gemv)]
                    g.replay()
                    ev0.record()
                    g.replay()
                    ev1.record()
                    ev1.synchronize()
                    t[with_gemv] = ev0.elapsed_time(ev1)
                best[mode] = min(best[mode], (t[True] - t[False]) * 1000.0 / args.reps)
        nbytes = n * k * 2
        for mode, us in best.items():
            print(json.dumps({"op": name, "m": args.m, "n": n, "k": k, "mode": mode, "us": round(us, 2),
                              "weight_tbps": round(nbytes / us / 1e6, 2)}), flush=True)
        del graphs, w


if __name__ == "__main__":
    main()
