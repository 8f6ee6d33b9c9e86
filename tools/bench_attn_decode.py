#!/usr/bin/env python3
"""Decode attention latency as a decode step sees it: hipGraph-replayed, K/V cold (a 512 MiB fill between calls
evicts L2 and the Infinity Cache, as the weight stream of a real step does). Time per call = (graph of R x
[fill, attention]) - (graph of R x [fill]) over R, min over rounds; impls interleaved in one process.

  python tools/bench_attn_decode.py --model llama3-70b --tp 8 --shapes 1x192 1x384 32x384 --impls 2 5

impl (ext.attn_set_impl / attn_set_v3_max_pairs): 2 = default dispatch; 3 = v3 (one workgroup per pair) forced;
5 = split small-batch kernel (v5) where it applies; 6 = v5 with the first merge (4 splits per load round);
7 = v4 (register ring, one split) forced; 9 = v2 (LDS-DMA ring, KPG 4, 2 slots) forced; 60 = v6 (matrix cores),
61 / 62 / 64 / 68 = v6 with 1 / 2 / 4 / 8 waves per (row, kv head) pair. Prints one JSON line per (shape, impl).
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


def set_impl(e, impl):
    e.attn_set_impl(2, 4096)
    # 60: the MFMA kernel (v6) with its default waves per pair; 61 / 62 / 64 / 68: v6 with 1 / 2 / 4 / 8 waves per pair
    # 600 + d: v6 at 2 waves per pair with ablation d (attn_set_v6_diag: 1 no compute, 2 no K loads, 4 no V DMAs)
    if hasattr(e, "attn_set_v6_diag"):
        e.attn_set_v6_diag(impl - 600 if 601 <= impl <= 607 else 0)
    if 601 <= impl <= 607:
        impl = 62
    e.attn_set_v6(2 if 60 <= impl <= 68 else 0)
    e.attn_set_v6_wpp(impl - 60 if 61 <= impl <= 68 else 0)
    e.attn_set_v3_max_pairs(4096)
    if impl in (7, 9):
        # the streaming kernels at any pair count, one split: 7 = v4 register ring, 9 = v2 (LDS-DMA ring)
        e.attn_set_impl(4 if impl == 9 else 2, 1)  # waves target 1 -> one split
        e.attn_set_impl(4 if impl == 9 else 2, -1)  # v2/v4 down to 1 pair
        e.attn_set_v3_max_pairs(0)
    if hasattr(e, "attn_set_v5_max_pairs"):
        e.attn_set_v5_max_pairs(4096 if impl in (5, 6) else (0 if impl in (3, 7, 9) else -1))
    if hasattr(e, "attn_set_v5_fold"):
        e.attn_set_v5_fold(4 if impl == 6 else (12 if impl == 5 else 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--shapes", nargs="+", default=["1x192", "1x384", "8x384", "32x384"], help="BxT (T = valid keys)")
    ap.add_argument("--cache-len", type=int, default=0, help="cache length (default: T)")
    ap.add_argument("--impls", type=int, nargs="+", default=[2, 1])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    e = ops.ext()
    cfg = get_preset(args.model)
    h, hkv, hd = cfg.num_attention_heads // args.tp, cfg.num_key_value_heads // args.tp, cfg.head_dim
    flush = torch.empty(512 << 18, dtype=torch.int32, device="cuda")  # 512 MiB
    for shape in args.shapes:
        b, t = (int(v) for v in shape.split("x"))
        tc = max(args.cache_len, t)
        g = torch.Generator(device="cuda").manual_seed(b * 7 + t)
        kc = torch.randn(b, hkv, tc, hd, device="cuda", generator=g).to(torch.bfloat16)
        vc = torch.randn(b, hkv, tc, hd, device="cuda", generator=g).to(torch.bfloat16)
        q = torch.randn(b, 1, h, hd, device="cuda", generator=g).to(torch.bfloat16)
        slot = torch.tensor([t - 1], dtype=torch.int32, device="cuda")
        ks = torch.zeros(b, dtype=torch.int32, device="cuda")
        res, first = {}, None
        graphs = {}
        for impl in args.impls:
            set_impl(e, impl)
            out = ops.attention(q, kc, vc, slot, ks)  # sizes the workspaces before capture
            torch.cuda.synchronize()
            first = out.float() if first is None else first
            diff = float((out.float() - first).abs().max())
            ga, gf = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                for _ in range(args.reps):
                    flush.fill_(1)
                    ops.attention(q, kc, vc, slot, ks)
            with torch.cuda.graph(gf):
                for _ in range(args.reps):
                    flush.fill_(1)
            graphs[impl] = (ga, gf, diff)
        set_impl(e, 2)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = {impl: float("inf") for impl in args.impls}
        for _ in range(args.rounds):
            for impl in args.impls:
                ga, gf, _ = graphs[impl]
                tt = []
                for gr in (ga, gf):
                    gr.replay()
                    ev0.record()
                    gr.replay()
                    ev1.record()
                    ev1.synchronize()
                    tt.append(ev0.elapsed_time(ev1))
                best[impl] = min(best[impl], (tt[0] - tt[1]) * 1000.0 / args.reps)
        for impl in args.impls:
            res = {"op": "attn_decode_graph", "model": args.model, "tp": args.tp, "b": b, "t": t, "cache_len": tc,
                   "impl": impl, "us": round(best[impl], 2), "max_diff_vs_first": round(graphs[impl][2], 5)}
            print(json.dumps(res), flush=True)
        del graphs, kc, vc


if __name__ == "__main__":
    main()
