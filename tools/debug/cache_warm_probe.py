#!/usr/bin/env python3
"""Decode GEMV (M = 1) time with its weights cold (rotated past the Infinity Cache), L2-warm (the same copy back to
back) and MALL-warm (the same copy, a 64 MiB streaming copy between calls to push it out of the 32 MiB of L2; the
copy's own time subtracted). Tells whether prefetching the next projection's weights during a latency-bound kernel
can pay. Usage: python tools/debug/cache_warm_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402
from jax_llama_amd.models.weights import PackedLinear  # noqa: E402

DEV = "cuda"


def timed(fn, iters=200):
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(iters):
        fn(i)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    e = ops.ext()
    src = torch.empty(64 << 18, device=DEV)  # 64 MiB
    dst = torch.empty_like(src)
    wsp = torch.empty(1 << 20, device=DEV)  # (split variants only; 0 / 6 do not read it)
    tk = torch.zeros(4096, device=DEV, dtype=torch.int32)
    for n, k in [(8192, 1024), (8192, 3584), (1280, 8192), (14336, 8192)]:
        copies = max(2, int((1 << 30) // (n * k * 2)) + 1)
        ws = [PackedLinear.from_dense((torch.randn(n, k, device=DEV) * 0.02).to(torch.bfloat16), DEV).weight
              for _ in range(copies)]
        x = torch.randn(1, k, device=DEV).to(torch.bfloat16)
        out = torch.empty(1, n, device=DEV, dtype=torch.bfloat16)
        for variant in (0, 6):
            def run(i, w=None):
                e.linear_skinny(x, w if w is not None else ws[i % copies], n, k, out, ops.MODE_STORE, -1.0, 0,
                                variant, wsp, tk)
            cold = timed(run)
            warm = timed(lambda i: run(i, ws[0]))
            cp = timed(lambda i: dst.copy_(src))
            mall = timed(lambda i: (dst.copy_(src), run(i, ws[0]))) - cp
            print(json.dumps({"n": n, "k": k, "variant": variant, "cold_us": round(cold, 2), "l2_warm_us": round(warm, 2),
                              "mall_warm_us": round(mall, 2), "copy_us": round(cp, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
