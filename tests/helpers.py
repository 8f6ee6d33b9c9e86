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


def gpu_meta_state_dict(cfg: LLaMAConfig, seed: int, emb_std: float = 1.0, std: float = 0.02,
                        device: str = "cuda") -> dict:
    """Random Meta-layout state dict generated on the GPU (fast at real model dims), bf16 values. Norm weights
    1 + 0.1 noise so the folded norms are exercised."""
    g = torch.Generator(device=device).manual_seed(seed)
    d, hd, f, v = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.vocab_size
    hq, hkv = cfg.num_attention_heads * hd, cfg.num_key_value_heads * hd

    def rnd(*shape, s=std):
        return (torch.randn(*shape, generator=g, device=device) * s).to(torch.bfloat16)

    def norm():
        return (1.0 + 0.1 * torch.randn(d, generator=g, device=device)).to(torch.bfloat16)

    sd = {"tok_embeddings.weight": rnd(v, d, s=emb_std), "norm.weight": norm(), "output.weight": rnd(v, d)}
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}."
        sd[p + "attention.wq.weight"] = rnd(hq, d)
        sd[p + "attention.wk.weight"] = rnd(hkv, d)
        sd[p + "attention.wv.weight"] = rnd(hkv, d)
        sd[p + "attention.wo.weight"] = rnd(d, hq)
        sd[p + "feed_forward.w1.weight"] = rnd(f, d)
        sd[p + "feed_forward.w2.weight"] = rnd(d, f, s=std / 2)
        sd[p + "feed_forward.w3.weight"] = rnd(f, d)
        sd[p + "attention_norm.weight"] = norm()
        sd[p + "ffn_norm.weight"] = norm()
    return sd


def argmax_gap(oracle, seq: torch.Tensor, mask: torch.Tensor, start: int) -> float:
    """Teacher-forced oracle logits over ``seq``: for every token from ``start`` on, (max logit - its logit) relative
    to the row's logit scale. 0 wherever the token is the oracle's argmax; a near-tie broken the other way costs at
    most the rounding error of the logits."""
    full_mask = torch.cat([mask, torch.ones(mask.shape[0], seq.shape[1] - mask.shape[1], dtype=mask.dtype)], 1)
    full_pos = full_mask.cumsum(-1) - 1
    lf = oracle.forward(seq, full_mask, full_pos).float()
    prev = lf[:, start - 1:-1]
    chosen = prev.gather(-1, seq[:, start:].long().to(prev.device).unsqueeze(-1)).squeeze(-1)
    return float(((prev.max(-1).values - chosen) / prev.abs().amax(-1)).max())
