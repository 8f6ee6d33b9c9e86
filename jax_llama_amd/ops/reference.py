"""Pure-PyTorch reference implementations of every fused op.

These are (a) the CPU execution path of the framework (used by CPU tests, the gloo
multi-rank tests and the JAX-CPU-equivalent "plumbing" config) and (b) the numerics oracle
the HIP kernels are tested against. Each function reproduces the *rounding points* of the
corresponding kernel (bf16 operands, fp32 accumulation) so CPU and GPU runs agree to
bf16 rounding.

Reference semantics being reproduced (``/root/reference/jax_llama/model.py``):
  * RMSNorm ``x * rsqrt(mean(x^2) + eps) * w``                        (:28-48)
  * interleaved (complex-pair) RoPE                                  (:50-92)
  * causal + padding masked softmax attention with a KV cache        (:169-291)
  * SwiGLU ``w2(silu(w1 x) * w3 x)``                                  (:337-340)
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


# ----------------------------------------------------------------------------------
# Weight packing (MFMA fragment layout, see ops/linear.py for the rationale)
# ----------------------------------------------------------------------------------
def pack_frag16x32(w: torch.Tensor) -> torch.Tensor:
    """Pack a row-major ``[N, K]`` weight into the 16x16x32-MFMA B-fragment layout.

    ``P[nt, ks, lane, e] = W[16*nt + (lane & 15), 32*ks + 8*(lane >> 4) + e]`` so one
    wave's 64 x 16-byte fragment load of a 16(n) x 32(k) block is 1 KiB contiguous.
    """
    n, k = w.shape
    assert n % 16 == 0 and k % 32 == 0, (n, k)
    return (w.reshape(n // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
            .reshape(n // 16, k // 32, 64, 8))


def pack_act(x: torch.Tensor, rows: int) -> torch.Tensor:
    """Packed-layout copy of a decode activation ``x [M, K]`` (csrc/kernels/common.h pack_off): rows zero-padded to
    ``rows`` (a multiple of 16), then the weights' fragment order; returned as ``[rows, K]`` (flat order
    ``[rows/16][K/32][64][8]``)."""
    m, k = x.shape
    xp = torch.zeros(rows, k, dtype=x.dtype, device=x.device)
    xp[:m] = x
    return pack_frag16x32(xp).reshape(rows, k)


def unpack_act(p: torch.Tensor, m: int) -> torch.Tensor:
    """Inverse of ``pack_act`` (first ``m`` rows)."""
    rows, k = p.shape
    return unpack_frag16x32(p.reshape(rows // 16, k // 32, 64, 8), rows, k)[:m]


def unpack_frag16x32(p: torch.Tensor, n: int, k: int) -> torch.Tensor:
    return (p.reshape(n // 16, k // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).contiguous()
            .reshape(n, k))


# ----------------------------------------------------------------------------------
# Elementwise / normalisation
# ----------------------------------------------------------------------------------
def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table[ids.long().clamp(0, table.shape[0] - 1)].float()


def inv_rms(x: torch.Tensor, eps: float) -> torch.Tensor:
    x = x.float()
    return torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)


def rms_scale(x: torch.Tensor, eps: float) -> torch.Tensor:
    """``bf16(x * rsqrt(mean(x^2)+eps))`` — the norm weight is folded into the next GEMM."""
    return (x.float() * inv_rms(x, eps)).to(BF16)


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """Un-fused RMSNorm exactly as the reference module (fp32 math)."""
    return x.float() * inv_rms(x, eps) * weight.float()


# ----------------------------------------------------------------------------------
# Linear layers (x @ W^T with W stored [N, K]); fp32 accumulate over bf16 operands
# ----------------------------------------------------------------------------------
def _mm(x: torch.Tensor, w_dense: torch.Tensor, rms_eps: Optional[float]) -> torch.Tensor:
    y = x.to(BF16).float() @ w_dense.float().t()
    if rms_eps is not None:
        y = y * inv_rms(x, rms_eps)
    return y


def linear(x, w_dense, rms_eps=None, out_dtype=BF16):
    return _mm(x, w_dense, rms_eps).to(out_dtype)


def linear_residual(x, w_dense, residual, rms_eps=None, accumulate=True):
    y = _mm(x, w_dense, rms_eps)
    if accumulate:
        residual.add_(y)
    else:
        residual.copy_(y)
    return residual


def linear_swiglu(x, w_dense_interleaved, rms_eps=None):
    """``w_dense_interleaved`` rows are 16-row tiles alternating gate (w1) / up (w3)."""
    y = _mm(x, w_dense_interleaved, rms_eps)
    m, n2 = y.shape
    y = y.reshape(m, n2 // 32, 2, 16)
    g, u = y[:, :, 0, :], y[:, :, 1, :]
    return (F.silu(g) * u).reshape(m, n2 // 2).to(BF16)


def interleave_gate_up(w1: torch.Tensor, w3: torch.Tensor) -> torch.Tensor:
    f, k = w1.shape
    assert f % 16 == 0
    return torch.stack([w1.reshape(f // 16, 16, k), w3.reshape(f // 16, 16, k)], 1).reshape(2 * f, k)


# ----------------------------------------------------------------------------------
# RoPE (interleaved pairs) + KV cache write
# ----------------------------------------------------------------------------------
def _llama31_scale(freqs: torch.Tensor) -> torch.Tensor:
    """Llama-3.1 ``use_scaled_rope`` frequency remap (factor 8, low/high 1/4, 8192 ctx)."""
    factor, low, high, old_ctx = 8.0, 1.0, 4.0, 8192.0
    wavelen = 2 * math.pi / freqs
    smooth = (old_ctx / wavelen - low) / (high - low)
    mid = (1 - smooth) * freqs / factor + smooth * freqs
    out = torch.where(wavelen < old_ctx / high, freqs, mid)
    return torch.where(wavelen > old_ctx / low, freqs / factor, out)


def rope_table(head_dim: int, end: int, theta: float, scaled: bool = False) -> torch.Tensor:
    """fp32 ``[end, head_dim/2, 2]`` (cos, sin) table (reference ``precompute_freqs_cis``,
    computed in fp64 and rounded once; the reference never stores it in bf16)."""
    i = torch.arange(0, head_dim, 2, dtype=torch.float64)[: head_dim // 2]
    freqs = 1.0 / (theta ** (i / head_dim))
    if scaled:
        freqs = _llama31_scale(freqs)
    t = torch.arange(end, dtype=torch.float64)
    ang = torch.outer(t, freqs)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()


def apply_rope(x: torch.Tensor, table: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
    """x: [M, nh, Dh]; positions: [M] (clamped into the table like the kernel)."""
    pos = positions.reshape(-1).long().clamp(0, table.shape[0] - 1)
    cs = table[pos]  # [M, Dh/2, 2]
    c, s = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    xr, xi = xf[..., 0], xf[..., 1]
    out = torch.stack([xr * c - xi * s, xr * s + xi * c], -1)
    return out.reshape(x.shape)


def rope_kv_write(qkv, table, positions, k_cache, v_cache, slot0: int, seq_len: int,
                  n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    """Split fused qkv ``[B*S, (H+2Hkv)*Dh]``, rotate q and k, store k/v at cache slots
    ``slot0 .. slot0+S-1`` of ``[B, Hkv, T, Dh]`` caches. Returns rotated q ``[B*S, H, Dh]``."""
    m = qkv.shape[0]
    b = m // seq_len
    q = qkv[:, : n_heads * head_dim].reshape(m, n_heads, head_dim)
    k = qkv[:, n_heads * head_dim:(n_heads + n_kv_heads) * head_dim].reshape(m, n_kv_heads, head_dim)
    v = qkv[:, (n_heads + n_kv_heads) * head_dim:].reshape(m, n_kv_heads, head_dim)
    qr = apply_rope(q, table, positions).to(BF16)
    kr = apply_rope(k, table, positions).to(BF16)
    kr = kr.reshape(b, seq_len, n_kv_heads, head_dim).permute(0, 2, 1, 3)
    vv = v.reshape(b, seq_len, n_kv_heads, head_dim).permute(0, 2, 1, 3)
    k_cache[:, :, slot0:slot0 + seq_len] = kr.to(k_cache.dtype)
    v_cache[:, :, slot0:slot0 + seq_len] = vv.to(v_cache.dtype)
    return qr


def linear_qkv_rope(x, w_dense, rms_eps, table, positions, k_cache, v_cache, slot0: int, seq_len: int,
                    n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    """Fused-kernel rounding points: fp32 projection -> fp32 RoPE -> one bf16 rounding."""
    y = _mm(x, w_dense, rms_eps)  # fp32 [M, (H+2Hkv)*Dh]
    m = y.shape[0]
    b = m // seq_len
    hq, hk = n_heads * head_dim, n_kv_heads * head_dim
    q = apply_rope(y[:, :hq].reshape(m, n_heads, head_dim), table, positions).to(BF16)
    k = apply_rope(y[:, hq:hq + hk].reshape(m, n_kv_heads, head_dim), table, positions)
    v = y[:, hq + hk:].reshape(m, n_kv_heads, head_dim)
    k_cache[:, :, slot0:slot0 + seq_len] = k.reshape(b, seq_len, n_kv_heads, head_dim).permute(0, 2, 1, 3).to(
        k_cache.dtype)
    v_cache[:, :, slot0:slot0 + seq_len] = v.reshape(b, seq_len, n_kv_heads, head_dim).permute(0, 2, 1, 3).to(
        v_cache.dtype)
    return q


# ----------------------------------------------------------------------------------
# Attention over the cache
# ----------------------------------------------------------------------------------
def attention(q, k_cache, v_cache, slot0: int, kv_start: torch.Tensor,
              key_mask: Optional[torch.Tensor] = None, return_weights: bool = False):
    """q: [B, S, H, Dh] (already rotated) for cache slots ``slot0+s``; caches
    ``[B, Hkv, T, Dh]``. Query at slot i attends keys j with ``kv_start[b] <= j <= i`` and
    ``key_mask[b, j]`` (if given). Rows with no valid key produce 0. Returns
    ``[B, S, H*Dh]`` bf16 (and fp32 weights ``[B, H, S, slot0+S]`` if requested)."""
    bsz, s, h, dh = q.shape
    hkv = k_cache.shape[1]
    rep = h // hkv
    t_len = slot0 + s
    k = k_cache[:, :, :t_len].float().repeat_interleave(rep, dim=1)  # [B,H,T,Dh]
    v = v_cache[:, :, :t_len].float().repeat_interleave(rep, dim=1)
    qf = q.float().permute(0, 2, 1, 3)  # [B,H,S,Dh]
    scores = qf @ k.transpose(-1, -2) / math.sqrt(dh)  # [B,H,S,T]
    qi = torch.arange(slot0, slot0 + s, device=q.device)[:, None]
    kj = torch.arange(t_len, device=q.device)[None, :]
    valid = (kj <= qi)[None]  # [1,S,T]
    valid = valid & (kj[None] >= kv_start.long().reshape(bsz, 1, 1))
    if key_mask is not None:
        valid = valid & key_mask[:, None, :t_len].bool()
    valid = valid[:, None]  # [B,1,S,T]
    scores = scores.masked_fill(~valid, float("-inf"))
    mx = scores.amax(-1, keepdim=True)
    mx = torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))
    p = torch.exp(scores - mx)
    denom = p.sum(-1, keepdim=True)
    p = torch.where(denom > 0, p / denom.clamp_min(1e-30), torch.zeros_like(p))
    out = (p @ v).permute(0, 2, 1, 3).reshape(bsz, s, h * dh).to(BF16)
    if return_weights:
        return out, p
    return out


# ----------------------------------------------------------------------------------
# Sampling (HF FlaxGenerationMixin semantics: temperature -> top-k -> top-p -> categorical)
# ----------------------------------------------------------------------------------
def argmax(logits: torch.Tensor) -> torch.Tensor:
    return logits.float().argmax(-1).to(torch.int32)  # first max index, like jnp.argmax


def top_k_top_p_filter(logits: torch.Tensor, temperature: float, top_k: int, top_p: float) -> torch.Tensor:
    """Returns warped logits with filtered entries at -inf (FlaxTemperature/TopK/TopP)."""
    x = logits.float()
    if temperature is not None and temperature != 1.0:
        x = x / temperature
    if top_k is not None and top_k != 0:
        k = min(top_k, x.shape[-1])
        vals, idx = torch.topk(x, k, dim=-1)
        y = torch.full_like(x, float("-inf"))
        x = y.scatter(-1, idx, vals)
    if top_p is not None and top_p < 1.0:
        vals, idx = torch.sort(x, dim=-1, descending=True)
        cum = torch.softmax(vals, -1).cumsum(-1)
        keep = cum < top_p
        keep = torch.roll(keep, 1, dims=-1)
        keep[:, 0] = True
        vals = torch.where(keep, vals, torch.full_like(vals, float("-inf")))
        x = torch.full_like(x, float("-inf")).scatter(-1, idx, vals)
    return x


def philox4x32_10(counter, key):
    """Philox4x32-10 (Salmon et al., SC'11) on uint32 numpy arrays: ``counter`` [..., 4], ``key``
    [2]. Bit-exact twin of ``philox4x32_10`` in csrc/kernels/topk_sample.hip."""
    import numpy as np
    c = [np.asarray(counter[..., i], dtype=np.uint64) for i in range(4)]
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    m0, m1, mask = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0, p1 = m0 * c[0], m1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c = [(hi1 ^ c[1] ^ k0) & mask, lo1, (hi0 ^ c[3] ^ k1) & mask, lo0]
        k0 = (k0 + np.uint64(0x9E3779B9)) & mask
        k1 = (k1 + np.uint64(0xBB67AE85)) & mask
    return np.stack([x.astype(np.uint32) for x in c], -1)


def topk_sorted(logits: torch.Tensor, k: int):
    """Top-k values (descending) and indices, ties broken by the lower index (lax.top_k order)."""
    import numpy as np
    x = logits.float().cpu().numpy()
    vals, idxs = [], []
    for row in x:
        order = np.lexsort((np.arange(row.size), -row))[:k]
        vals.append(row[order])
        idxs.append(order)
    return torch.from_numpy(np.stack(vals)), torch.from_numpy(np.stack(idxs).astype(np.int32))


def topk_sample(logits: torch.Tensor, k: int, temperature: float, top_p: float, seed: int, step: int) -> torch.Tensor:
    """Reference of the on-device sampler: temperature -> top-k -> top-p (HF keep rule) ->
    Gumbel-max with Philox(seed; counter = (rank-in-top-k, row, step, 0))."""
    import numpy as np
    vals, idx = topk_sorted(logits, k)
    v = vals.numpy().astype(np.float32) / np.float32(temperature)
    p = np.exp(v - v[:, :1])
    p = p / p.sum(-1, keepdims=True)
    excl = np.cumsum(p, -1) - p
    keep = excl < np.float32(top_p)
    keep[:, 0] = True
    b = v.shape[0]
    ctr = np.zeros((b, k, 4), dtype=np.uint32)
    ctr[..., 0] = np.arange(k, dtype=np.uint32)[None]
    ctr[..., 1] = np.arange(b, dtype=np.uint32)[:, None]
    ctr[..., 2] = np.uint32(step)
    r = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))[..., 0]
    u = ((r >> 8).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)
    g = -np.log(-np.log(u))
    score = np.where(keep, v + g, -np.inf)
    choice = score.argmax(-1)
    return idx[torch.arange(b), torch.from_numpy(choice)].to(torch.int32)
