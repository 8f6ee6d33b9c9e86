#!/usr/bin/env python3
"""Text generation entry point -- the MI355X counterpart of the reference ``jax_example.py``.

Same ``load()`` / ``main()`` surface (``jax_example.py:10-40``): build the tensor-parallel layout,
the tokenizer (SentencePiece for LLaMA-1/2, tiktoken-format BPE for Llama-3), load the Meta
checkpoint and run the two fixed prompts through ``LLaMA.generate_from_str``. Differences by
design: one process per GPU (launch with ``torchrun --nproc-per-node MP``; TP degree = world size,
like the reference's ``(1, n_devices)`` mesh), each rank reads only its own slices of the
checkpoint, argparse instead of ``fire`` (not installed), and a ``--synthetic`` mode that runs a
random-init model of a named architecture with synthetic prompt ids (no checkpoint needed).

  python examples/generate.py --ckpt_dir /ckpt/8B --tokenizer_path /ckpt/tokenizer.model --is_llama3
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/generate.py --ckpt_dir /ckpt/70B ...
  python examples/generate.py --synthetic --model llama3-8b --max_gen_len 32
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_llama_amd import LLaMA, LLaMA2Tokenizer, LLaMA3Tokenizer, LLaMAForCausalLM  # noqa: E402
from jax_llama_amd.parallel import TPComm, init_distributed  # noqa: E402
from jax_llama_amd.parallel.partition import Mesh  # noqa: E402
from jax_llama_amd.utils.checkpoint import load_meta_rank  # noqa: E402

PROMPTS = ["The capital of Germany is the city of",
           "Here is my sonnet in the style of Shakespeare about an artificial intelligence:"]


def load(ckpt_dir: str, tokenizer_path: str, is_llama3: bool, max_seq_len: int = 2048, **model_kwargs) -> LLaMA:
    """Reference ``load`` (jax_example.py:10-31) on the MI355X runtime."""
    ctx = init_distributed()
    ctx.setup_mesh(tp=ctx.world)
    with open(os.path.join(ckpt_dir, "params.json")) as f:
        hidden = int(json.load(f)["dim"])
    comm = TPComm.from_context(ctx, fused_hidden=hidden)
    tokenizer = LLaMA3Tokenizer(tokenizer_path) if is_llama3 else LLaMA2Tokenizer(tokenizer_path)
    params, config = load_meta_rank(ckpt_dir, tokenizer, ctx.tp_rank, ctx.tp_size, max_seq_len=max_seq_len)
    config.bos_token_id, config.eos_token_id = tokenizer.bos_id, tokenizer.eos_id
    model = LLaMAForCausalLM(config, device=ctx.device, comm=comm, _do_init=False, **model_kwargs).load_params(params, sharded=True)
    del params
    return LLaMA(None, model, tokenizer, mesh=Mesh(dp=1, mp=ctx.tp_size, rank=ctx.rank))


def main(ckpt_dir: str, tokenizer_path: str, is_llama3: bool, max_gen_len: int = 256, temperature: float = 0.8,
         top_p: float = 0.95):
    """Reference ``main`` (jax_example.py:33-40)."""
    generator = load(ckpt_dir, tokenizer_path, is_llama3)
    results = generator.generate_from_str(PROMPTS, max_gen_len=max_gen_len, temperature=temperature, top_p=top_p)
    if int(os.environ.get("RANK", "0")) == 0:
        for result in results:
            print(result)
            print("\n==================================\n")
    return results


def synthetic(model_name: str, batch: int, prompt_len: int, max_gen_len: int, temperature: float, top_p: float):
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.runtime.engine import GenerationConfig
    ctx = init_distributed()
    ctx.setup_mesh(tp=ctx.world)
    cfg = get_preset(model_name, max_seq_len=max(2048, prompt_len + max_gen_len))
    comm = TPComm.from_context(ctx, fused_hidden=cfg.hidden_size)
    model = LLaMAForCausalLM(cfg, device=ctx.device, comm=comm, _do_init=False).init_random(seed=0)
    toks = torch.randint(3, cfg.vocab_size, (batch, prompt_len), generator=torch.Generator().manual_seed(0),
                         dtype=torch.int32)
    gc = GenerationConfig(max_length=prompt_len + max_gen_len, do_sample=temperature != 0.0,
                          temperature=temperature, top_p=top_p, pad_token_id=0, eos_token_id=-1)
    t0 = time.perf_counter()
    seq = model.generate(toks, generation_config=gc).sequences
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    dt = time.perf_counter() - t0
    if ctx.rank == 0:
        print(f"{model_name}: {batch} x {max_gen_len} tokens in {dt:.3f} s "
              f"({batch * max_gen_len / dt:.1f} tok/s incl. prefill + graph capture)")
        print("first row:", seq[0, prompt_len:prompt_len + 16].tolist())


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ckpt_dir")
    ap.add_argument("--tokenizer_path")
    ap.add_argument("--is_llama3", action="store_true")
    ap.add_argument("--max_gen_len", type=int, default=256)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top_p", type=float, default=0.95)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--prompt_len", type=int, default=16)
    a = ap.parse_args()
    if a.synthetic:
        synthetic(a.model, a.batch, a.prompt_len, a.max_gen_len, a.temperature, a.top_p)
    else:
        if not (a.ckpt_dir and a.tokenizer_path):
            ap.error("--ckpt_dir and --tokenizer_path are required (or use --synthetic)")
        main(a.ckpt_dir, a.tokenizer_path, a.is_llama3, a.max_gen_len, a.temperature, a.top_p)
