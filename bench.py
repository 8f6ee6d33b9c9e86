#!/usr/bin/env python3
"""Headline benchmark: output tokens/s of LLaMA generation on MI355X (BASELINE.json metric).

One *step* = one full ``generate`` call on a batch of synthetic prompts: bf16 prefill of
``--prompt-len`` tokens, then ``--gen-len`` hipGraph-replayed greedy decode steps (EOS disabled so
every row produces every token; all work — prefill, every layer, lm_head, sampler, state update —
is inside the timed region). Weights are random-init with the exact architecture of ``--model``
(no checkpoints are available offline); the data are synthetic token ids.

Multi-GPU (torchrun, one process per GPU, RCCL): the world is split into ``world / tp``
data-parallel replicas of a ``tp``-way tensor-parallel model (default tp = 1: each GPU serves its
own batch -> weak scaling). ``value`` = total output tokens of all replicas / max-over-ranks time.

  python bench.py --gpus 1 --steps 3 --warmup 1
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --model llama3-70b --tp 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    # Serving-throughput operating point: 2048 concurrent sequences per replica (KV cache 103 GB of the
    # 288 GB HBM; ~44 ms per decode step = ~22 tokens/s per sequence; 35.1k tok/s vs 33.5k at 1024 and
    # 33.6k at 1536 -- profiles/README.md). Smaller batches are latency points (decode_ms_per_token):
    # --batch 1 / 16 / 512 / 1024.
    ap.add_argument("--batch", type=int, default=2048, help="sequences per replica")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--layers", type=int, default=None, help="debug only: override layer count (INVALID for the metric)")
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel import TPComm, init_distributed
    from jax_llama_amd.runtime.engine import GenerationConfig, get_engine

    ctx = init_distributed()
    world = ctx.world
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ctx.setup_mesh(tp=args.tp)
    comm = TPComm.from_context(ctx)
    dev = ctx.device
    overrides = {} if args.layers is None else {"num_hidden_layers": args.layers}
    max_len = args.prompt_len + args.gen_len
    cfg = get_preset(args.model, max_seq_len=max(2048, max_len), **overrides)
    model = LLaMAForCausalLM(cfg, device=dev, comm=comm).init_random(seed=1234)
    torch.cuda.synchronize(dev)

    gen = torch.Generator().manual_seed(100 + ctx.dp_rank)
    prompts = torch.randint(3, cfg.vocab_size, (args.batch, args.prompt_len), generator=gen, dtype=torch.int32)
    gc = GenerationConfig(max_length=max_len, do_sample=False, pad_token_id=0, eos_token_id=-1)

    def step():
        return model.generate(prompts, generation_config=gc).sequences

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ctx.barrier()
    torch.cuda.synchronize(dev)

    # decode-only timing (prefill excluded) on the already-captured engine: one extra run
    eng = get_engine(model, args.batch, max_len)
    torch.cuda.synchronize(dev)
    tp0 = time.perf_counter()
    eng.prefill_only(prompts, None, gc)
    torch.cuda.synchronize(dev)
    ttft = time.perf_counter() - tp0

    elapsed, ttft = ctx.all_reduce_max([elapsed, ttft])
    replicas = world // args.tp
    out_tokens = replicas * args.batch * args.gen_len * args.steps
    value = out_tokens / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    decode_ms_per_token = (ms_step - 1000.0 * ttft) / max(1, args.gen_len - 1)
    res = {
        "metric": "output_tokens_per_sec",
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak" if args.tp == 1 else "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic token ids, random-init weights (no checkpoints offline)",
        "config": {
            "model": args.model + ("" if args.layers is None else f"-{args.layers}L-DEBUG"),
            "global_batch": replicas * args.batch,
            "seq_len": max_len,
            "prompt_len": args.prompt_len,
            "gen_len": args.gen_len,
            "parallelism": f"dp{replicas}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
            "mp": args.tp,
        },
        "ttft_ms": round(1000.0 * ttft, 3),
        "decode_ms_per_token": round(decode_ms_per_token, 4),
        "decode_tokens_per_sec": round(replicas * args.batch * 1000.0 / decode_ms_per_token, 2),
        "weight_gb_per_gpu": round(model.weight_bytes() / 1e9, 3),
        "hbm_roofline_ms_per_token": round(model.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4),
        "decode_kernel_choice": {f"m{k[0]}_n{k[1]}_k{k[2]}_mode{k[3]}": v
                                 for k, v in __import__("jax_llama_amd.ops.autotune", fromlist=["x"]).table().items()},
        "gemm_plan_choice": {f"m{k[0]}_n{k[1]}_k{k[2]}": f"ks{v[0]}_tile{v[1]}" for k, v in
                             __import__("jax_llama_amd.ops.autotune", fromlist=["x"]).ksplit_table().items()},
    }
    if ctx.rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    del out


if __name__ == "__main__":
    main()
