#!/usr/bin/env python3
"""Timeline of the fused small-batch decode launch (csrc/kernels/gemv.hip qkv_attn_kernel) at the Llama-3-70B
tensor-parallel shard's shapes: every workgroup stamps the wall clock (100 MHz) at its phase boundaries
(qkv_attn_set_stamps), weights cold (a 512 MiB fill before each launch). Prints, per role, the phase times in
microseconds after the first workgroup started (median over --reps launches of the per-launch min / max):

  qkv:  start, GEMV + epilogue done (1), published (2)
  attn: start, wait over (1), step computed (2), output written (3), o go flags set (4, last one only)
  o:    start, go seen (1), MFMAs done (2), epilogue done (3)

and the graph-timed launch: fused with o vs fused without o + the standalone o GEMV.

  python tools/qkv_attn_timeline.py --batch 1 --keys 256 --tp-exchange
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402
from jax_llama_amd.models.weights import PackedLinear  # noqa: E402
from jax_llama_amd.ops import reference as ref  # noqa: E402

DEV = "cuda"
BF16 = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--keys", type=int, default=256, help="valid keys (cache slot = keys - 1)")
    ap.add_argument("--cache", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tp-exchange", action="store_true", help="o epilogue: the TP granule exchange (world-1 instance)")
    ap.add_argument("--o-nt", type=int, default=2)
    args = ap.parse_args()
    e = ops.ext()
    b, d, h, hkv, dh, k = args.batch, 8192, 8, 1, 128, 8192
    n = (h + 2 * hkv) * dh
    g = torch.Generator(device=DEV).manual_seed(0)
    wq = PackedLinear.random(n, k, DEV, 0.02, g)
    wo = PackedLinear.random(d, h * dh, DEV, 0.02, g)
    x = (torch.randn(b, k, device=DEV, generator=g) * 0.5).to(BF16)
    table = ref.rope_table(dh, 4096, 500000.0).to(DEV)
    slot = args.keys - 1
    pos = torch.full((b,), slot, dtype=torch.int32, device=DEV)
    sl = torch.tensor([slot], dtype=torch.int32, device=DEV)
    kc = torch.randn(b, hkv, args.cache, dh, device=DEV, generator=g).to(BF16)
    vc = torch.randn(b, hkv, args.cache, dh, device=DEV, generator=g).to(BF16)
    kv_start = torch.zeros(b, dtype=torch.int32, device=DEV)
    hres = torch.zeros(b, d, device=DEV)
    hb = torch.empty(b, d, dtype=BF16, device=DEV)
    car = None
    state = 0
    if args.tp_exchange:
        from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
        car = CustomAllReduce.local(max_bytes=CustomAllReduce.fused_bytes(d))
        state = car._live()
    e.qkv_attn_set_o_nt(args.o_nt)
    og = e.qkv_attn_o_groups(b, h // hkv, d, h * dh)
    cus = ops._num_cus(x.device)
    splits = e.qkv_attn_splits(b, b, hkv, h // hkv, args.cache, n, cus, 2, og)
    assert splits > 0 and og > 0, (splits, og)
    flush = torch.empty(512 << 18, dtype=torch.int32, device=DEV)

    def fused(with_o):
        o = (wo, hres, hb, None, state) if with_o else None
        return ops.linear_qkv_attention(x, wq, 1e-5, table, pos, kc, vc, sl, kv_start, h, hkv, dh, splits, spl=2, o=o)

    def unfused():
        a = fused(False)
        if args.tp_exchange:
            ops.linear_tp_residual(a, wo, hres, hb, state)
        else:
            ops.linear_residual(a, wo, hres, mirror=hb)

    fused(True)
    unfused()
    torch.cuda.synchronize()
    grid_q = (n // 16) * 2
    grid_a = b * hkv * splits
    grid = grid_q + grid_a + og
    stamps = torch.zeros(grid * 8, dtype=torch.int64, device=DEV)
    roles = {"qkv": (0, grid_q, 3), "attn": (grid_q, grid_q + grid_a, 5), "o": (grid_q + grid_a, grid, 4)}
    per = {r: [[] for _ in range(2 * nphase)] for r, (_, _, nphase) in roles.items()}
    e.qkv_attn_set_stamps(stamps)
    try:
        for _ in range(args.reps):
            flush.fill_(1)
            stamps.zero_()
            torch.cuda.synchronize()
            fused(True)
            torch.cuda.synchronize()
            s = stamps.view(grid, 8).cpu()
            t0 = int(s[:, 0].min())
            for r, (lo, hi, nphase) in roles.items():
                for i in range(nphase):
                    col = s[lo:hi, i]
                    col = col[col > 0]
                    if col.numel() == 0:
                        continue
                    per[r][2 * i].append((int(col.min()) - t0) / 100.0)
                    per[r][2 * i + 1].append((int(col.max()) - t0) / 100.0)
    finally:
        e.qkv_attn_set_stamps(None)
    out = {"batch": b, "keys": args.keys, "splits": splits, "grid": [grid_q, grid_a, og],
           "o_epilogue": "tp_exchange" if args.tp_exchange else "residual"}
    for r, (_, _, nphase) in roles.items():
        out[r] = {f"p{i}": [round(statistics.median(per[r][2 * i]), 2) if per[r][2 * i] else None,
                            round(statistics.median(per[r][2 * i + 1]), 2) if per[r][2 * i + 1] else None]
                  for i in range(nphase)}
    print(json.dumps(out), flush=True)

    # graph-timed: fused with o vs fused without o + the standalone o GEMV (weights cold)
    res = {}
    for name, fn in (("fused_o", lambda: fused(True)), ("fused_then_o", unfused)):
        ga, gf = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga):
            for _ in range(args.reps):
                flush.fill_(1)
                fn()
        with torch.cuda.graph(gf):
            for _ in range(args.reps):
                flush.fill_(1)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(3):
            tt = []
            for gr in (ga, gf):
                gr.replay()
                ev0.record()
                gr.replay()
                ev1.record()
                ev1.synchronize()
                tt.append(ev0.elapsed_time(ev1))
            best = min(best, (tt[0] - tt[1]) * 1000.0 / args.reps)
        res[name] = round(best, 2)
    print(json.dumps({"graph_us": res}), flush=True)
    e.qkv_attn_set_o_nt(2)
    if car is not None:
        car.close()


if __name__ == "__main__":
    main()
