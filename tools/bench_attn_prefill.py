#!/usr/bin/env python3
"""Prefill attention throughput (causal, GQA) at real model shapes: TFLOP/s of impl 2 (the default dispatch of the
GQA-shared 32x32x16 MFMA flash kernel, 32 queries per wave), 7 / 8 (pipelined / unpipelined, 4 waves), 9 / 13
(pipelined, 8 waves; 13 with asm LDS-DMA and interleaved next-tile scores) and impl 1 (v1). FLOPs counted for the causal triangle only:
4 * B * H * Dh * S (S + 1) / 2. Prints one JSON line per (shape, impl)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402

SHAPES = [  # (name, B, S, H, Hkv)
    ("8b_b1_s2048", 1, 2048, 32, 8), ("8b_b16_s2048", 16, 2048, 32, 8), ("8b_b1_s8192", 1, 8192, 32, 8),
    ("8b_b2048_s128", 2048, 128, 32, 8), ("70b_b1_s2048", 1, 2048, 64, 8), ("7b_b16_s2048", 16, 2048, 32, 32),
]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default=None, help="run only this shape name (profiling)")
    ap.add_argument("--impl", type=int, default=None, help="run only this impl (profiling)")
    ap.add_argument("--impls", type=int, nargs="*", default=None, help="impls to compare (default 2 7 8 9 13 1)")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    e = ops.ext()
    for name, b, s, h, hkv in SHAPES:
        if args.shape and name != args.shape:
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        kc = torch.randn(b, hkv, s, 128, device="cuda", generator=g).to(torch.bfloat16)
        vc = torch.randn(b, hkv, s, 128, device="cuda", generator=g).to(torch.bfloat16)
        q = torch.randn(b, s, h, 128, device="cuda", generator=g).to(torch.bfloat16)
        ks = torch.zeros(b, dtype=torch.int32, device="cuda")
        slot = torch.zeros(1, dtype=torch.int32, device="cuda")
        flops = 4.0 * b * h * 128 * s * (s + 1) / 2
        ref = None
        impls = [i for i in (args.impls or (2, 7, 8, 9, 13, 1)) if not (i == 1 and s * s * b * h > 2048 * 2048 * 16 * 32)
                 and (args.impl is None or i == args.impl)]
        best, diffs = {i: float("inf") for i in impls}, {}
        for impl in impls:  # warm-up + correctness vs the first impl
            e.attn_prefill_set_impl(impl)
            o = ops.attention(q, kc, vc, slot, ks)
            torch.cuda.synchronize()
            diffs[impl] = 0.0 if ref is None else float((o.float() - ref.float()).abs().max())
            ref = o if ref is None else ref
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(args.rounds):  # interleaved rounds, min per impl (DVFS drift between impls)
            for impl in impls:
                e.attn_prefill_set_impl(impl)
                n = 5
                ev[0].record()
                for _ in range(n):
                    ops.attention(q, kc, vc, slot, ks)
                ev[1].record()
                torch.cuda.synchronize()
                best[impl] = min(best[impl], ev[0].elapsed_time(ev[1]) * 1000 / n)
        for impl in impls:
            us = best[impl]
            print(json.dumps({"shape": name, "impl": impl, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                              "max_diff_vs_first": round(diffs[impl], 5)}), flush=True)
        e.attn_prefill_set_impl(2)
        del kc, vc, q
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
