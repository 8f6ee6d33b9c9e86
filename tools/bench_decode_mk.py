#!/usr/bin/env python3
"""A/B of the persistent decode step (csrc/kernels/decode_mk.hip) against the per-layer kernels: decode ms/token over
the full generation window (runtime/benchmark.py decode_latency), interleaved rounds, one JSON line per point.

  python tools/bench_decode_mk.py --model llama3-8b --batches 1 4 --rounds 2
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=256)
    args = ap.parse_args()
    import torch

    from jax_llama_amd import ops
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.runtime.benchmark import decode_latency

    kw = {} if args.layers is None else {"num_hidden_layers": args.layers}
    cfg = get_preset(args.model, max_seq_len=max(2048, args.prompt_len + args.gen_len), **kw)
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=1)
    for rnd in range(args.rounds):
        for b in args.batches:
            for mk in (True, False):
                ops.DECODE_MK = mk
                p = decode_latency(model, b, args.prompt_len, args.gen_len, seed=7)
                p.update({"model": args.model, "layers": cfg.num_hidden_layers, "decode_mk": mk, "round": rnd,
                          "mk_error": ops.decode_mk_error("cuda") if mk else 0})
                print(json.dumps(p), flush=True)


if __name__ == "__main__":
    main()
