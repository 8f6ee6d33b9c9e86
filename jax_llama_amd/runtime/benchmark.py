"""Measurement helpers shared by ``bench.py`` and ``tools/``: decode latency points (hipGraph-replayed
decode steps timed with HIP events, prefill excluded) and end-to-end generate throughput.

BASELINE.md's protocol: decode tokens/s = B x generated tokens / decode wall time, hipGraph replay,
prefill excluded; prompts of 128 synthetic tokens, max_gen_len 256, B in {1, 8, 32}, greedy.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .engine import DecodeEngine, GenerationConfig


def synthetic_prompts(vocab: int, batch: int, prompt_len: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(3, vocab, (batch, prompt_len), generator=g, dtype=torch.int32)


def decode_latency(model, batch: int, prompt_len: int = 128, gen_len: int = 256, steps: int = 64,
                   seed: int = 0, barrier=None, do_sample: bool = False) -> Dict[str, float]:
    """Prefill ``batch`` prompts into a ``prompt_len + gen_len`` cache (``prefill_ms``: the second, warm prefill; the
    first autotunes), then time ``steps`` replays of
    the captured decode step (every layer, lm_head, sampler, state update). Every rank of a TP group
    must call this with the same arguments (the step contains the TP collectives)."""
    assert steps + 2 < gen_len, "replays must stay inside the cache"
    max_len = prompt_len + gen_len
    eng = DecodeEngine(model, batch, max_len, use_graph=True)
    gc = GenerationConfig(max_length=max_len, do_sample=do_sample, temperature=0.8, top_p=0.95, top_k=50,
                          pad_token_id=0, eos_token_id=-1)
    eng.gc = gc
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    eng.prefill(prompts, None)  # cold: autotunes new prefill shapes and grows the workspaces; not timed
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    eng.prefill(prompts, None)  # warm prefill: ``prefill_ms``
    ev1.record()
    eng._decode_step()  # eager step: sizes the workspaces before capture
    eng._ensure_graph()
    eng._graph.replay()
    torch.cuda.synchronize(dev)
    ttft_ms = ev0.elapsed_time(ev1)
    if barrier is not None:
        barrier()
    ev0.record()
    for _ in range(steps):
        eng._graph.replay()
    ev1.record()
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / steps
    model.comm.check()
    del eng
    return {"batch": batch, "decode_ms_per_token": round(ms, 4),
            "decode_tokens_per_sec": round(batch * 1000.0 / ms, 2), "prefill_ms": round(ttft_ms, 3)}


def time_to_first_token(model, batch: int, prompt_len: int, reps: int = 3, seed: int = 0,
                        barrier=None) -> Dict[str, float]:
    """Prefill of ``batch`` synthetic prompts of ``prompt_len`` tokens up to the first generated token
    (every layer's GEMMs + flash attention + KV-cache writes, last-position lm_head, greedy argmax),
    timed with HIP events after one warm-up prefill (autotune, workspace growth). Median of ``reps``."""
    eng = DecodeEngine(model, batch, prompt_len + 8, use_graph=False)
    gc = GenerationConfig(max_length=prompt_len + 8, do_sample=False, pad_token_id=0, eos_token_id=-1)
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    eng.prefill_only(prompts, None, gc)
    torch.cuda.synchronize(dev)
    if barrier is not None:
        barrier()
    times = []
    for _ in range(reps):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        eng.prefill_only(prompts, None, gc)
        ev1.record()
        torch.cuda.synchronize(dev)
        times.append(ev0.elapsed_time(ev1))
    model.comm.check()
    del eng
    ms = sorted(times)[len(times) // 2]
    return {"batch": batch, "prompt_len": prompt_len, "ttft_ms": round(ms, 3),
            "prefill_tokens_per_sec": round(batch * prompt_len * 1000.0 / ms, 1)}


def generate_tokens_per_sec(model, batch: int, prompt_len: int, gen_len: int, gc: GenerationConfig,
                            seed: int = 0, reps: int = 1, barrier=None) -> Dict[str, float]:
    """Whole ``generate`` calls (prefill + every decode step + sampler), output tokens per second."""
    import time
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    model.generate(prompts, generation_config=gc)  # warm-up: engine, capture, autotune
    torch.cuda.synchronize(dev)
    if barrier is not None:
        barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        model.generate(prompts, generation_config=gc)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"batch": batch, "ms_per_generate": round(1000 * dt, 2), "tokens_per_sec": round(batch * gen_len / dt, 2)}
