"""Shared test helpers: tiny configs, random Meta weights, model construction."""
from __future__ import annotations

import torch

from jax_llama_amd.config import LLaMAConfig
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.utils.checkpoint import meta_state_dict_to_params, random_meta_state_dict
from oracle import OracleLLaMA


def tiny_config(**kw) -> LLaMAConfig:
    """jax_test.py:28-41 fixture: dim 32, 4 layers, 4 heads, 2 kv heads, vocab 256."""
    base = dict(vocab_size=256, hidden_size=32, intermediate_size=96, num_hidden_layers=4,
                num_attention_heads=4, num_key_value_heads=2, max_sequence_length=64, rms_norm_eps=1e-5)
    base.update(kw)
    return LLaMAConfig(**base)


def gpu_config(**kw) -> LLaMAConfig:
    """Smallest config the GPU kernels accept (head_dim 128, N%16, K%32)."""
    base = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                num_attention_heads=2, num_key_value_heads=1, max_sequence_length=256, rms_norm_eps=1e-5)
    base.update(kw)
    return LLaMAConfig(**base)


def build(config: LLaMAConfig, device="cpu", seed=0, comm=None):
    sd = random_meta_state_dict(config, seed=seed)
    params = meta_state_dict_to_params(sd, config.num_hidden_layers)
    model = LLaMAForCausalLM(config, device=device, comm=comm, _do_init=False).load_params(params)
    oracle = OracleLLaMA(sd, config.num_hidden_layers, config.num_attention_heads,
                         config.num_key_value_heads, config.rms_norm_eps, config.rope_theta)
    return model, oracle, sd, params


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def left_padded_batch(lengths, s, vocab, pad, seed=0):
    g = torch.Generator().manual_seed(seed)
    b = len(lengths)
    toks = torch.full((b, s), pad, dtype=torch.int32)
    mask = torch.zeros(b, s, dtype=torch.int32)
    for i, n in enumerate(lengths):
        toks[i, s - n:] = torch.randint(3, vocab, (n,), generator=g, dtype=torch.int32)
        mask[i, s - n:] = 1
    return toks, mask
