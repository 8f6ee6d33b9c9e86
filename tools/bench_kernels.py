#!/usr/bin/env python3
"""Micro-benchmark of the decode hot kernels at real model shapes (one MI355X).

Weights rotate over enough copies (> 2x the 256 MiB Infinity Cache) that every timed call streams
from HBM, as in a real decode step. Prints one JSON line per (op, shape, variant) with
microseconds and effective TB/s. Usage: python tools/bench_kernels.py [--model llama3-8b] [--m 1 16]
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
from jax_llama_amd.ops import reference as ref  # noqa: E402

DEV = "cuda"


def timeit(fn, iters=30):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(iters):
        fn(i)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000.0 / iters


def copies_for(nbytes):
    return max(2, int((600 << 20) // max(nbytes, 1)) + 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16])
    ap.add_argument("--variants", type=int, nargs="+", default=[1, 6])
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ops", nargs="+", default=None, help="subset of qkv o gate_up down lm_head attn")
    ap.add_argument("--attn-impls", default="2:4096,4:4096", help="impl:waves_target pairs for attn A/B")
    ap.add_argument("--attn-shapes", nargs="*", default=None, help="BxT decode attention shapes (default: a sweep)")
    ap.add_argument("--v3-kpg", type=int, nargs="*", default=[0],
                    help="small-batch decode attention (v3) chunk-depth multipliers to sweep (0: by size, the default)")
    args = ap.parse_args()
    args.attn_impls = [tuple(int(v) for v in p.split(":")) for p in args.attn_impls.split(",")]
    cfg = get_preset(args.model)
    d, f, hd = cfg.hidden_size, cfg.intermediate_size // args.tp, cfg.head_dim
    h, hkv = cfg.num_attention_heads // args.tp, cfg.num_key_value_heads // args.tp
    shapes = {
        # activations are the bf16 mirror of the residual stream in the model (every projection input)
        "qkv": ((h + 2 * hkv) * hd, d, torch.bfloat16, ops.MODE_QKV),
        "o": (d, h * hd, torch.bfloat16, ops.MODE_RESIDUAL),
        "gate_up": (2 * f, d, torch.bfloat16, ops.MODE_SWIGLU),
        "down": (d, f, torch.bfloat16, ops.MODE_RESIDUAL),
        "lm_head": (cfg.vocab_size // args.tp, d, torch.bfloat16, ops.MODE_STORE),
    }
    e = ops.ext()
    for name, (n, k, xdt, mode) in shapes.items():
        if args.ops and name not in args.ops:
            continue
        nbytes = n * k * 2
        ws = [PackedLinear.random(n, k, DEV) for _ in range(copies_for(nbytes))]
        for m in args.m:
            x = torch.randn(m, k, device=DEV).to(xdt)
            for var in args.variants:
                ops.GEMV_VARIANT = var
                # packed-x variants read a real packed copy of x (ref.pack_act), as in the model
                xpk = ref.pack_act(x, ops.packed_rows(m)) if var in ops.XP_VARIANTS else None
                ops._SK_SIZES.clear()
                if mode == ops.MODE_QKV:
                    table = torch.randn(4096, hd // 2, 2, device=DEV)
                    pos = torch.zeros(m, dtype=torch.int32, device=DEV)
                    kc = torch.zeros(m, hkv, 512, hd, dtype=torch.bfloat16, device=DEV)
                    vc = torch.zeros_like(kc)
                    slot = torch.zeros(1, dtype=torch.int32, device=DEV)

                    def fn(i, x=x, table=table, pos=pos, kc=kc, vc=vc, slot=slot, xpk=xpk):
                        ops.linear_qkv_rope(x, ws[i % len(ws)], 1e-5, table, pos, kc, vc, slot, 1, h, hkv, hd,
                                            x_packed=xpk)
                elif mode == ops.MODE_RESIDUAL:
                    out = torch.zeros(m, n, device=DEV)

                    def fn(i, x=x, out=out, xpk=xpk):
                        ops.linear_residual(x, ws[i % len(ws)], out, x_packed=xpk)
                elif mode == ops.MODE_SWIGLU:
                    def fn(i, x=x, xpk=xpk):
                        ops.linear_swiglu(x, ws[i % len(ws)], rms_eps=1e-5, x_packed=xpk)
                else:
                    out32 = torch.empty(m, n, device=DEV)

                    def fn(i, x=x, xpk=xpk, out32=out32):
                        ops._gpu_linear(x, ws[i % len(ws)], out32, ops.MODE_STORE, 1e-5, True, None, xpk)
                us = timeit(fn)
                ops._SK_SIZES.clear()
                print(json.dumps({"op": name, "n": n, "k": k, "m": m, "variant": var, "us": round(us, 2),
                                  "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
        del ws
        torch.cuda.empty_cache()
    ops.GEMV_VARIANT = 0
    # decode attention at the bench shape
    if args.ops and "attn" not in args.ops:
        return
    ap_shapes = ((16, 384), (1, 4096), (64, 1024), (256, 384), (512, 384), (512, 256), (1024, 384), (2048, 128),
                 (2048, 256), (2048, 384))
    for b, t in ap_shapes if not args.attn_shapes else [tuple(int(v) for v in p.split("x")) for p in args.attn_shapes]:
        kc = torch.randn(b, hkv, t, hd, device=DEV).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(b, 1, h, hd, device=DEV).to(torch.bfloat16)
        slot = torch.tensor([t - 1], dtype=torch.int32, device=DEV)
        ks = torch.zeros(b, dtype=torch.int32, device=DEV)
        nbytes = 2 * kc.numel() * 2
        ref_out = None
        for (impl, target), kpg in [(it, kk) for it in args.attn_impls for kk in args.v3_kpg]:
            e.attn_set_diag(1 if impl >= 100 else 0)  # 100 + impl: diagnostic stream-only run of impl
            impl = impl % 100
            e.attn_set_impl(impl, target)
            e.attn_set_v3_kpg(kpg)
            e.attn_set_v3_max_pairs(4096)
            us = timeit(lambda i: ops.attention(q, kc, vc, slot, ks))
            o = ops.attention(q, kc, vc, slot, ks).float()
            ref_out = o if ref_out is None else ref_out
            print(json.dumps({"op": "attn_decode", "impl": impl, "waves_target": target, "v3_kpg": kpg, "b": b, "t": t,
                              "nsplit": e.attn_decode_splits(b, hkv, t, h // hkv), "us": round(us, 2),
                              "TBps": round(nbytes / us / 1e6, 3),
                              "max_diff_vs_first": round(float((o - ref_out).abs().max()), 5)}), flush=True)
        e.attn_set_diag(0)
        e.attn_set_impl(2, 4096)
        e.attn_set_v3_kpg(0)
        e.attn_set_v3_max_pairs(4096)
        del kc, vc


if __name__ == "__main__":
    main()
