#!/usr/bin/env python3
"""Time to first token (prefill of a synthetic prompt + first greedy token) of a random-init model.

  python tools/ttft.py --model llama3-8b --batch 1 --prompt-len 128 512 2048 8192
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
    ap.add_argument("--prompt-len", type=int, nargs="+", default=[2048])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.runtime.benchmark import time_to_first_token
    cfg = get_preset(args.model, max_seq_len=max(args.prompt_len) + 16)
    m = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=1)
    for b in args.batch:
        for s in args.prompt_len:
            r = time_to_first_token(m, b, s, reps=args.reps)
            r["model"] = args.model
            line = json.dumps(r)
            print(line, flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(line + "\n")
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
