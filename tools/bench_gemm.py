#!/usr/bin/env python3
"""Tiled MFMA GEMM (csrc/kernels/gemm.hip) vs the vendor library (torch.mm -> hipBLASLt) on the
Llama projection shapes, for decode batches (M = 64..512) and prefill (M = B * S).

Weights rotate over copies larger than the Infinity Cache so each timed call reads them from HBM.
Prints one JSON line per (shape, impl): microseconds, TFLOP/s and weight TB/s.
Usage: python tools/bench_gemm.py [--m 128 256 4096] [--model llama3-8b] [--ksplit 0]
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


def timeit(fn, iters):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(iters):
        fn(i)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--m", type=int, nargs="+", default=[64, 128, 256, 512, 4096])
    ap.add_argument("--ksplit", type=int, nargs="+", default=[0], help="0 = library heuristic")
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--impl", type=int, nargs="+", default=[2], help="label of the round (the tiled kernel is gemm2/gemm4)")
    ap.add_argument("--ops", nargs="+", default=None)
    ap.add_argument("--rounds", type=int, default=1, help="interleaved A/B rounds of the impl list (one process)")
    ap.add_argument("--tile", type=int, nargs="+", default=[0], help="gemm2 tile config(s): 0 auto, 1 256x256, "
                    "2 128x256, 3 128x128")
    ap.add_argument("--mode", default="store", choices=["store", "swiglu", "residual"],
                    help="epilogue (the model's: qkv/lm_head store, gate_up swiglu, o/down residual)")
    ap.add_argument("--rms", action="store_true", help="fused RMSNorm statistic (store / swiglu)")
    ap.add_argument("--g5-diag", type=int, nargs="+", default=[0], help="gemm5 ablation bits (wrong results): 1 no "
                    "MFMAs, 2 weights from a cached zero fragment, 4 x from a cached stage")
    ap.add_argument("--group", type=int, nargs="+", default=[0], help="gemm4 tile rasterisation: m-tiles per launch "
                    "group (gemm_set_g4_group; 0 = by shape)")
    ap.add_argument("--tp", type=int, default=1, help="per-rank shapes of that TP degree (qkv / gate_up column-parallel, "
                    "o / down row-parallel, lm_head vocab-parallel; parallel/partition.py)")
    ap.add_argument("--data", default="normal", choices=["normal", "uniform"],
                    help="operand distribution (uniform: as tools/debug/gemm4w_probe.hip)")
    args = ap.parse_args()
    mode = {"store": 0, "residual": 1, "swiglu": 2}[args.mode]
    eps = 1e-5 if args.rms and mode != 1 else -1.0
    cfg = get_preset(args.model)
    d, f, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    h, hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    tp = args.tp
    shapes = {"qkv": ((h + 2 * hkv) * hd // tp, d), "o": (d, h * hd // tp), "gate_up": (2 * f // tp, d),
              "down": (d, f // tp), "lm_head": (cfg.vocab_size // tp // 16 * 16, d)}
    e = ops.ext()
    for name, (n, k) in shapes.items():
        if args.ops and name not in args.ops:
            continue
        nbytes = n * k * 2
        copies = max(2, int((700 << 20) // nbytes) + 1)
        if args.data == "uniform":
            dense = [((torch.rand(n, k, device=DEV) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(copies)]
        else:
            dense = [(torch.randn(n, k, device=DEV) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        packed = [PackedLinear.from_dense(w, DEV) for w in dense]
        for m in args.m:
            if args.data == "uniform":
                x = (torch.rand(m, k, device=DEV) * 2 - 1).to(torch.bfloat16)
            else:
                x = (torch.randn(m, k, device=DEV)).to(torch.bfloat16)
            out = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
            if mode == 1:
                out = torch.zeros(m, n, device=DEV, dtype=torch.float32)
                mir = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
            elif mode == 2:
                out = torch.empty(m, n // 2, device=DEV, dtype=torch.bfloat16)
            flop = 2.0 * m * n * k
            iters = max(5, min(200, int(2e13 / flop)))
            res = {}
            ref = None
            first = {}
            for rnd, impl in [(r, i) for r in range(args.rounds) for i in args.impl]:
                for ks in args.ksplit:
                 for diag, grp in [(d, g) for d in args.g5_diag for g in args.group]:
                  e.gemm5_set_diag(diag)
                  e.gemm_set_g4_group(grp)
                  for tile in args.tile:
                    kk = ks or e.gemm_ksplit(m, n, k)
                    if tile in (16, 17) and kk > 1 and eps > 0:
                        continue  # (gemm4 256 x 128 / 192: no K split under the fused norm)
                    if kk > 1 and (k // 32) // kk < 4 and tile not in (11, 12):
                        continue
                    if tile in (11, 12) and (k % 64 or (k // 64) // kk < 1):
                        continue
                    ws = torch.empty(max(1, kk * m * (n + 1)), device=DEV, dtype=torch.float32)
                    tcfg = tile
                    rws = torch.empty(m, device=DEV) if (eps > 0 and kk == 1 and tile not in (11, 12)) else None

                    def run(i, kk=kk, ws=ws, tile=tcfg, rws=rws):
                        e.gemm(x, packed[i % copies].weight, n, k, out, mode, True, mir if mode == 1 else None, kk,
                               ws if (kk > 1 or tile in (11, 12)) else None, eps, tile, None, rws)
                    res[f"v{impl}_ks{kk}_t{tile}" + (f"_diag{diag}" if diag else "") + (f"_g{grp}" if grp else "")  + "" +
                        (f"_r{rnd}" if args.rounds > 1 else "")] = timeit(run, iters)
                    run(0)
                    if mode != 0 or (diag & 255):  # (numerics of the other epilogues: tests/test_gemm4_gpu.py)
                        continue
                    got = out.float()
                    if ref is None:
                        xs = x.float()
                        if eps > 0:
                            xs = xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + eps)
                        ref = (xs @ dense[0].float().t())
                    err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                    assert err < 2e-2 or (tile >= 50 and (tile - 50) & 14), (name, m, impl, kk, err)
                    if impl >= 2 and tile < 5:  # gemm2 pipeline variants must agree bit for bit (same per-accumulator order)
                        f0 = first.setdefault((kk, tile), got.clone())
                        assert torch.equal(f0, got), ("variant mismatch", name, m, impl, kk, tile)
            e.gemm5_set_diag(0)
            e.gemm_set_g4_group(0)
            if not args.no_blas and mode == 0:
                res["hipblaslt"] = timeit(lambda i: torch.mm(x, dense[i % copies].t(), out=out), iters)
            for impl, us in res.items():
                print(json.dumps({"op": name, "m": m, "n": n, "k": k, "impl": impl, "us": round(us, 2),
                                  "tflops": round(flop / us / 1e6, 1), "weight_tbps": round(nbytes / us / 1e6, 2)}),
                      flush=True)
        del dense, packed
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
