#!/usr/bin/env python3
"""CU-partition probe: decode attention and a GEMM on disjoint CU sets (CU-masked streams, csrc/kernels/placement.hip).

1. census: how the mask bits map onto XCDs / CUs (distinct CUs a 4096-workgroup launch touches per mask);
2. attention (Llama-3-8B, half batch M = 1024 rows, 256 keys) alone on the first k CUs of the mask order;
3. the GEMM (--op, tile --tile) alone on the other 256 - k CUs, and on all CUs;
4. both at once on the two masked streams.

One JSON line per k: ``both_us`` (the two sides at once) against ``serial_all_us`` (each alone on the whole chip, in
sequence).

  python tools/cu_partition_probe.py --k 64 96 128 160
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter

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


def mask_words(bits, ncu):
    w = [0] * ((ncu + 31) // 32)
    for b in bits:
        w[b // 32] |= 1 << (b % 32)
    return w


def census(e, stream, blocks=4096):
    out = torch.zeros(2 * blocks, dtype=torch.int32, device=DEV)
    with torch.cuda.stream(stream):
        e.cu_census(out)
    torch.cuda.synchronize()
    v = out.view(-1, 2).cpu().tolist()
    cus = set()
    per_xcc = Counter()
    for hw, xcc in v:
        hw &= 0xFFFFFFFF
        key = (xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)
        if key not in cus:
            per_xcc[xcc & 0xF] += 1
        cus.add(key)
    return len(cus), dict(sorted(per_xcc.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--t", type=int, default=384)
    ap.add_argument("--keys", type=int, default=256)
    ap.add_argument("--op", default="gate_up", choices=["gate_up", "down", "o", "qkv"])
    ap.add_argument("--tile", type=int, default=7)
    ap.add_argument("--k", type=int, nargs="+", default=[64, 96, 128, 160])
    ap.add_argument("--census-only", action="store_true")
    args = ap.parse_args()
    e = ops.ext()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    full = torch.cuda.current_stream()
    print(json.dumps({"census": "default stream", "cus": census(e, full)}), flush=True)

    cfg = get_preset(args.model)
    d, f, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    h, hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    m = args.m
    n, k, mode = {"gate_up": (2 * f, d, 2), "down": (d, f, 1), "o": (d, h * hd, 1), "qkv": ((h + 2 * hkv) * hd, d, 0)}[
        args.op]
    if not args.census_only:
        w = PackedLinear.from_dense((torch.randn(n, k, device=DEV) * 0.02).to(torch.bfloat16), DEV)
        x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
        out = (torch.empty(m, n // 2, device=DEV, dtype=torch.bfloat16) if mode == 2 else
               torch.zeros(m, n, device=DEV, dtype=torch.float32) if mode == 1 else
               torch.empty(m, n, device=DEV, dtype=torch.bfloat16))
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

        def gemm():
            e.gemm(x, w.weight, n, k, out, mode, True, mir, 1, None, eps, args.tile, None, rws if eps > 0 else None)

        ta_all = timed(attn)
        tg_all = timed(gemm)
        print(json.dumps({"attn_all_us": round(ta_all, 1), "gemm_all_us": round(tg_all, 1), "op": args.op,
                          "tile": args.tile}), flush=True)
    for kk in args.k:
        sa = torch.cuda.ExternalStream(e.cu_mask_stream(mask_words(range(kk), ncu)))
        sg = torch.cuda.ExternalStream(e.cu_mask_stream(mask_words(range(kk, ncu), ncu)))
        rec = {"k": kk, "census_attn_side": census(e, sa), "census_gemm_side": census(e, sg)}
        if not args.census_only:
            def both():
                cur = torch.cuda.current_stream()
                sa.wait_stream(cur)
                sg.wait_stream(cur)
                with torch.cuda.stream(sa):
                    attn()
                with torch.cuda.stream(sg):
                    gemm()
                cur.wait_stream(sa)
                cur.wait_stream(sg)

            def attn_k():
                cur = torch.cuda.current_stream()
                sa.wait_stream(cur)
                with torch.cuda.stream(sa):
                    attn()
                cur.wait_stream(sa)

            def gemm_rest():
                cur = torch.cuda.current_stream()
                sg.wait_stream(cur)
                with torch.cuda.stream(sg):
                    gemm()
                cur.wait_stream(sg)

            ta = timed(attn_k)
            tg = timed(gemm_rest)
            tb = timed(both)
            rec.update({"attn_k_us": round(ta, 1), "attn_k_tbps": round(m * hkv * args.keys * hd * 4 / ta / 1e6, 2),
                        "gemm_rest_us": round(tg, 1), "both_us": round(tb, 1),
                        "serial_all_us": round(ta_all + tg_all, 1)})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
