#!/usr/bin/env python3
"""One decode latency point (hipGraph-replayed steps, prefill excluded) of a synthetic model; the
unit to run under rocprofv3 for a per-kernel breakdown of small-batch decode.

  python tools/decode_point.py --model llama3-8b --batch 1 32 --steps 64
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, nargs="+", default=[1])
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--sample", action="store_true")
    ap.add_argument("--tp-proxy", type=int, default=1, help="> 1: ONE rank of that MP degree on this GPU "
                    "(parallel/comm.py TPRankProxyComm; bench.py tp_rank_proxy)")
    ap.add_argument("--tune-report", action="store_true", help="print the decode-kernel choices and the graph-timed "
                    "microseconds of every candidate measured (ops/autotune.py)")
    args = ap.parse_args()
    import torch
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.runtime.benchmark import decode_latency
    cfg = get_preset(args.model, max_seq_len=2048)
    comm = None
    if args.tp_proxy > 1:
        from jax_llama_amd.parallel import TPRankProxyComm
        comm = TPRankProxyComm.create(args.tp_proxy, fused_hidden=cfg.hidden_size)
    m = LLaMAForCausalLM(cfg, device="cuda", comm=comm, _do_init=False).init_random(seed=1)
    for b in args.batch:
        r = decode_latency(m, b, args.prompt_len, args.gen_len, steps=args.steps, do_sample=args.sample)
        r["model"] = args.model
        r["mp"] = args.tp_proxy
        r["fused_row_parallel"] = comm is not None and comm.fused is not None
        r["hbm_roofline_ms"] = round(m.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()
    if args.tune_report:
        from jax_llama_amd.ops import autotune
        for (m, n, k, _), t in autotune.measured().items():
            print(json.dumps({"tune": "gemv", "m": m, "n": n, "k": k, "us": t, "best": min(t, key=t.get)}), flush=True)


if __name__ == "__main__":
    main()
