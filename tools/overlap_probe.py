#!/usr/bin/env python3
"""Co-residency probe: does a half-batch decode attention launch overlap a half-batch GEMM launched on another stream?

Llama-3-8B shapes at the headline operating point split in two micro-batches (M = B = 1024 rows, cache of 384 slots,
256 keys per row): the GEMM (gate_up with the SwiGLU epilogue and fused norm, or down / o with the residual epilogue)
on tile config ``--tiles``, the decode attention (the default dispatch, or ``--attn-impl``). Times G alone, A alone,
and G || A (each order of launch) on two streams; prints one JSON line per (tile, order) with the overlap fraction
``(tG + tA - tGA) / min(tG, tA)`` (1 = the shorter one fully hidden, 0 = serialised).

  python tools/overlap_probe.py --tiles 16 17 14 7
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

DEV = "cuda"


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--t", type=int, default=384, help="cache slots")
    ap.add_argument("--keys", type=int, default=256)
    ap.add_argument("--op", default="gate_up", choices=["gate_up", "down", "o", "qkv"])
    ap.add_argument("--tiles", type=int, nargs="+", default=[16, 17, 14, 7])
    ap.add_argument("--attn-v", type=int, default=0, help="attn_set_v7 mode (0 = default dispatch)")
    ap.add_argument("--diag", action="store_true", help="attention: the stream-only build (no math; wrong results)")
    args = ap.parse_args()
    cfg = get_preset(args.model)
    d, f, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    h, hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    e = ops.ext()
    if args.attn_v and hasattr(e, "attn_set_v7"):
        e.attn_set_v7(args.attn_v)
    if args.diag:
        e.attn_set_diag(1)
    m = args.m
    n, k, mode = {"gate_up": (2 * f, d, 2), "down": (d, f, 1), "o": (d, h * hd, 1), "qkv": ((h + 2 * hkv) * hd, d, 0)}[
        args.op]
    w = PackedLinear.from_dense((torch.randn(n, k, device=DEV) * 0.02).to(torch.bfloat16), DEV)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    if mode == 2:
        out = torch.empty(m, n // 2, device=DEV, dtype=torch.bfloat16)
    elif mode == 1:
        out = torch.zeros(m, n, device=DEV, dtype=torch.float32)
    else:
        out = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    mir = torch.empty(m, n, device=DEV, dtype=torch.bfloat16) if mode == 1 else None
    eps = 1e-5 if mode != 1 else -1.0
    rws = torch.ones(m, device=DEV)

    kc = (torch.randn(m, hkv, args.t, hd, device=DEV) * 0.5).to(torch.bfloat16)
    vc = torch.randn(m, hkv, args.t, hd, device=DEV).to(torch.bfloat16)
    q = torch.randn(m, 1, h, hd, device=DEV).to(torch.bfloat16)
    slot = torch.tensor([args.keys - 1], dtype=torch.int32, device=DEV)
    kv_start = torch.zeros(m, dtype=torch.int32, device=DEV)

    def attn():
        ops.attention(q, kc, vc, slot, kv_start)

    side = torch.cuda.Stream()
    for tile in args.tiles:
        def gemm(tile=tile):
            e.gemm(x, w.weight, n, k, out, mode, True, mir, 1, None, eps, tile, None,
                   rws if eps > 0 else None)

        def par(first_g):
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            if first_g:
                gemm()
                with torch.cuda.stream(side):
                    attn()
            else:
                with torch.cuda.stream(side):
                    attn()
                gemm()
            main.wait_stream(side)

        try:
            tg = timed(gemm)
        except RuntimeError as ex:  # noqa: PERF203
            print(json.dumps({"tile": tile, "error": str(ex)[:200]}), flush=True)
            continue
        ta = timed(attn)
        tga = timed(lambda: par(True))
        tag = timed(lambda: par(False))
        for order, tb in (("gemm_first", tga), ("attn_first", tag)):
            print(json.dumps({"op": args.op, "m": m, "tile": tile, "keys": args.keys, "order": order, "diag": args.diag,
                              "gemm_us": round(tg, 1), "attn_us": round(ta, 1), "both_us": round(tb, 1),
                              "overlap": round((tg + ta - tb) / min(tg, ta), 3)}), flush=True)


if __name__ == "__main__":
    main()
