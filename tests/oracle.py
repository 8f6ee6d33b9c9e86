"""Independent fp32 pure-PyTorch LLaMA oracle, written from the model spec (Meta layout).

Meta's ``llama`` package (the reference's oracle, ``jax_test.py``) is not installable here, so
this file re-states its math directly: complex-number RoPE via ``torch.polar``, GQA by
``repeat_kv`` copies, an explicit causal + padding mask with the reference's ``finfo.min``
bias (``model.py:263-267``), ``[out, in]`` weights. It shares no code with the framework.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch


def precompute_freqs_cis(dim: int, end: int, theta: float = 10000.0) -> torch.Tensor:
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64)[: dim // 2] / dim))
    t = torch.arange(end, dtype=torch.float64)
    freqs = torch.outer(t, freqs)
    return torch.polar(torch.ones_like(freqs), freqs).to(torch.complex64)


def apply_rotary_emb(x: torch.Tensor, freqs_cis: torch.Tensor) -> torch.Tensor:
    """x: (B, S, H, Dh); freqs_cis: (B, S, Dh/2) complex."""
    xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2).contiguous())
    out = torch.view_as_real(xc * freqs_cis[:, :, None, :]).flatten(3)
    return out


def rmsnorm(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


class OracleLLaMA:
    def __init__(self, sd: Dict[str, torch.Tensor], n_layers: int, n_heads: int, n_kv_heads: int,
                 eps: float, rope_theta: float = 10000.0, max_len: int = 4096):
        self.sd = {k: v.float() for k, v in sd.items()}
        self.L, self.H, self.Hkv, self.eps = n_layers, n_heads, n_kv_heads, eps
        d = self.sd["tok_embeddings.weight"].shape[1]
        self.dh = d // n_heads
        self.freqs = precompute_freqs_cis(self.dh, max_len, rope_theta)

    def forward(self, tokens: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                position_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Full-sequence forward (no cache). Returns fp32 logits (B, S, V)."""
        sd = self.sd
        dev = sd["tok_embeddings.weight"].device  # runs where its weights are (CPU, or fp32 on the GPU)
        b, s = tokens.shape
        if attention_mask is None:
            attention_mask = torch.ones(b, s, dtype=torch.int64)
        if position_ids is None:
            position_ids = torch.arange(s).expand(b, s)
        tokens, attention_mask, position_ids = tokens.to(dev), attention_mask.to(dev), position_ids.to(dev)
        if self.freqs.device != dev:
            self.freqs = self.freqs.to(dev)
        h = sd["tok_embeddings.weight"][tokens.long()]
        fc = self.freqs[position_ids.long().clamp(min=0)]
        causal = torch.tril(torch.ones(s, s, dtype=torch.bool, device=dev))
        mask = causal[None, None] & attention_mask.bool()[:, None, None, :]
        bias = torch.where(mask, 0.0, torch.finfo(torch.float32).min)
        rep = self.H // self.Hkv
        for i in range(self.L):
            p = f"layers.{i}."
            x = rmsnorm(h, sd[p + "attention_norm.weight"], self.eps)
            q = (x @ sd[p + "attention.wq.weight"].t()).reshape(b, s, self.H, self.dh)
            k = (x @ sd[p + "attention.wk.weight"].t()).reshape(b, s, self.Hkv, self.dh)
            v = (x @ sd[p + "attention.wv.weight"].t()).reshape(b, s, self.Hkv, self.dh)
            q, k = apply_rotary_emb(q, fc), apply_rotary_emb(k, fc)
            k = k.repeat_interleave(rep, dim=2)
            v = v.repeat_interleave(rep, dim=2)
            sc = torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(self.dh) + bias
            pr = torch.softmax(sc, -1)
            o = torch.einsum("bhqk,bkhd->bqhd", pr, v).reshape(b, s, -1)
            h = h + o @ sd[p + "attention.wo.weight"].t()
            x = rmsnorm(h, sd[p + "ffn_norm.weight"], self.eps)
            g = torch.nn.functional.silu(x @ sd[p + "feed_forward.w1.weight"].t())
            u = x @ sd[p + "feed_forward.w3.weight"].t()
            h = h + (g * u) @ sd[p + "feed_forward.w2.weight"].t()
        h = rmsnorm(h, sd["norm.weight"], self.eps)
        return h @ sd["output.weight"].t()

    def greedy(self, tokens: torch.Tensor, attention_mask: torch.Tensor, max_len: int,
               pad: int, eos: int) -> torch.Tensor:
        """HF greedy loop re-implemented naively (full recompute each step)."""
        b, s = tokens.shape
        seq = torch.full((b, max_len), pad, dtype=torch.int64)
        seq[:, :s] = tokens
        mask = torch.ones(b, max_len, dtype=torch.int64)
        mask[:, :s] = attention_mask
        pos = (mask.cumsum(-1) - 1)
        finished = torch.zeros(b, dtype=torch.bool)
        cur = s
        while cur < max_len and not bool(finished.all()):
            logits = self.forward(seq[:, :cur], mask[:, :cur], pos[:, :cur])[:, -1]
            nxt = logits.argmax(-1)
            nxt = torch.where(finished, torch.full_like(nxt, pad), nxt)
            finished |= nxt == eos
            seq[:, cur] = nxt
            cur += 1
        return seq
