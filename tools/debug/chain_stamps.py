"""Diagnostic: one decode-chain launch at Llama-3-8B layer dims (M rows) against the four unchained launches it
replaces, CUDA-event timed (median of 30), plus the chain's per-workgroup wall-clock timeline
([start, waited, streamed, done] stamps, 100 MHz) summarised per stage.

  python tools/debug/chain_stamps.py [--m 1] [--json-out gpurun_out/chain_stamps.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402
from jax_llama_amd.models.weights import PackedLinear  # noqa: E402
from jax_llama_amd.ops import reference as ref  # noqa: E402

DEV, BF16 = "cuda", torch.bfloat16


def lin(n, k):
    return PackedLinear.from_dense((torch.randn(n, k) * 0.02).to(BF16), DEV)


def timed(fn, reps=30):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    m, d, f, nh, nkv, dh = args.m, 4096, 14336, 32, 8, 128
    wo, wgu, wd, wqkv = lin(d, d), lin(2 * f, d), lin(d, f), lin((nh + 2 * nkv) * dh, d)
    a = (torch.randn(m, d) * 0.5).to(BF16).to(DEV)
    h = torch.randn(m, d, device=DEV)
    hb = h.to(BF16)
    act = torch.empty(m, f, dtype=BF16, device=DEV)
    table = ref.rope_table(dh, 256, 500000.0).to(DEV)
    pos = torch.full((m,), 5, dtype=torch.int32, device=DEV)
    kc = torch.zeros(m, nkv, 64, dh, dtype=BF16, device=DEV)
    vc = torch.zeros_like(kc)
    slot = torch.tensor([5], dtype=torch.int32, device=DEV)
    st = ops.ChainState(1, DEV)
    qkv = (wqkv, table, pos, kc, vc, slot, 1, nh, nkv, dh)

    def chained(stamps=None):
        ops.chain_epoch_bump(st)
        ops.decode_chain(a, wo, wgu, wd, h, hb, act, 1e-5, st, 0, qkv, stamps=stamps)

    ops.GEMV_VARIANT = 1

    def unchained():
        ops.linear_residual(a, wo, h, mirror=hb)
        g = ops.linear_swiglu(hb, wgu, rms_eps=1e-5)
        ops.linear_residual(g, wd, h, mirror=hb)
        ops.linear_qkv_rope(hb, wqkv, 1e-5, table, pos, kc, vc, slot, 1, nh, nkv, dh)

    for _ in range(3):
        chained()
        unchained()
    torch.cuda.synchronize()
    res = {"m": m, "chain_us": timed(chained), "unchained_us": timed(unchained)}
    stamps = torch.zeros(4 * 4096, dtype=torch.int64, device=DEV)
    chained(stamps)
    torch.cuda.synchronize()
    st.check()
    s = stamps.view(-1, 4).cpu()
    counts = [d // 16, (2 * f // 16) // 2, d // 16, ((nh + 2 * nkv) * dh // 16) // 2]
    t0 = s[: sum(counts), 0].min().item()
    us = lambda v: round((v - t0) / 100.0, 2)  # noqa: E731  (100 MHz wall clock)
    stages, b = [], 0
    for name, c in zip(("wo", "w1w3", "w2", "wqkv"), counts):
        x = s[b: b + c]
        b += c
        wait = (x[:, 1] - x[:, 0]).float() / 100.0
        stream = (x[:, 2] - x[:, 1]).float() / 100.0
        stages.append({"stage": name, "wgs": c, "start_first": us(x[:, 0].min().item()),
                       "start_last": us(x[:, 0].max().item()), "waited_first": us(x[:, 1].min().item()),
                       "waited_last": us(x[:, 1].max().item()), "done_first": us(x[:, 3].min().item()),
                       "done_last": us(x[:, 3].max().item()), "wait_us_median": round(wait.median().item(), 2),
                       "stream_us_median": round(stream.median().item(), 2),
                       "stream_us_max": round(stream.max().item(), 2)})
    res["stages"] = stages
    line = json.dumps(res)
    print(line)
    if args.json_out:
        with open(args.json_out, "a") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
