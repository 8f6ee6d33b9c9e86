"""Persistent decode step (csrc/kernels/decode_mk.hip: every layer of one decode token for batch <= 4 in one launch):
against the per-layer kernels it replaces, the fp32 oracle, graph replay, and at the Llama-3-8B layer dims."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd import ops
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.models.llama import mask_to_kv_start
from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
from helpers import build, gpu_config, left_padded_batch, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _decode_once(model, toks, mask, mk: bool, monkeypatch):
    """Prefill ``toks`` then one greedy decode token with the persistent step on or off: (logits of the decode
    token, the final residual rows, the layer-0 K cache row written by the step)."""
    monkeypatch.setattr(ops, "DECODE_MK", mk)
    b, s = toks.shape
    cache = model.init_cache(b, s + 8)
    kv_start, key_mask = mask_to_kv_start(mask, DEV)
    assert key_mask is None
    pos = (mask.cumsum(-1) - 1).clamp_min(0).to(torch.int32).to(DEV)
    logits, _, _, _ = model.forward_tokens(toks.to(DEV), pos.reshape(-1), cache, 0, kv_start, None, logits_mode="last")
    cache.advance(s)
    nxt = logits.float().argmax(-1).to(torch.int32)
    pos1 = (pos[:, -1] + 1).to(torch.int32)
    l1, h1, _, _ = model.forward_tokens(nxt[:, None], pos1, cache, cache.index_t, kv_start, None,
                                         logits_mode="last")
    torch.cuda.synchronize()
    return l1.float().cpu(), h1.float().cpu(), cache.k[0, :, :, s].float().cpu(), nxt.cpu()


@pytest.mark.parametrize("lens", [[9], [4, 9, 7], [9, 9, 9, 9]])
def test_decode_mk_matches_layer_kernels_and_oracle(lens, monkeypatch):
    cfg = gpu_config(hidden_size=512, intermediate_size=1024, num_attention_heads=4, num_key_value_heads=2,
                     num_hidden_layers=3)
    _, oracle, _, params = build(cfg, seed=21)
    model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks, mask = left_padded_batch(lens, 9, cfg.vocab_size, pad=2, seed=22)
    monkeypatch.setattr(ops, "DECODE_MK", True)
    assert ops.decode_mk_ok(model, len(lens), 1, None)
    lm, hm, km, nxt = _decode_once(model, toks, mask, True, monkeypatch)
    assert ops.decode_mk_error(DEV) == 0
    ll, hl, kl, nxt2 = _decode_once(model, toks, mask, False, monkeypatch)
    assert torch.equal(nxt, nxt2)
    # same bf16 rounding points except the RMSNorm statistic's summation order
    assert rel_err(hm, hl) < 1e-2, rel_err(hm, hl)
    assert rel_err(lm, ll) < 2e-2, rel_err(lm, ll)
    assert rel_err(km, kl) < 1e-2
    # fp32 oracle over the whole sequence, last position
    full = torch.cat([toks, nxt[:, None]], 1)
    fmask = torch.cat([mask, torch.ones(len(lens), 1, dtype=mask.dtype)], 1)
    fpos = (fmask.cumsum(-1) - 1).clamp_min(0)
    lo = oracle.forward(full, fmask, fpos)[:, -1]
    assert rel_err(lm, lo) < 5e-2, rel_err(lm, lo)


def test_decode_mk_graph_replay_matches_eager(monkeypatch):
    monkeypatch.setattr(ops, "DECODE_MK", True)
    cfg = gpu_config(num_hidden_layers=2)
    _, _, _, params = build(cfg, seed=23)
    model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks, mask = left_padded_batch([5, 8], 8, cfg.vocab_size, pad=2, seed=24)
    gc = GenerationConfig(max_length=64, do_sample=False, pad_token_id=2, eos_token_id=-1)
    a = DecodeEngine(model, 2, 64, use_graph=True).run(toks, mask, gc).clone()
    b = DecodeEngine(model, 2, 64, use_graph=False).run(toks, mask, gc).clone()
    assert torch.equal(a, b)
    assert ops.decode_mk_error(DEV) == 0


def test_decode_mk_greedy_agrees_with_layer_kernels(monkeypatch):
    cfg = gpu_config(num_hidden_layers=2)
    _, _, _, params = build(cfg, seed=25)
    model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks, mask = left_padded_batch([3, 11, 6], 11, cfg.vocab_size, pad=2, seed=26)
    gc = GenerationConfig(max_length=80, do_sample=False, pad_token_id=2, eos_token_id=-1)
    monkeypatch.setattr(ops, "DECODE_MK", True)
    a = DecodeEngine(model, 3, 80, use_graph=True).run(toks, mask, gc).clone()
    monkeypatch.setattr(ops, "DECODE_MK", False)
    b = DecodeEngine(model, 3, 80, use_graph=True).run(toks, mask, gc).clone()
    agree = (a.long() == b.long()).float().mean().item()
    assert agree > 0.97, agree  # (near-ties may break the other way: the norm statistic sums in another order)


@pytest.mark.parametrize("batch", [1, 4])
def test_decode_mk_llama3_8b_dims(batch, monkeypatch):
    """Two layers at the real Llama-3-8B shapes (GQA rep 4, K = 14336 staging, multi-tile wave runs): the step's
    residual and logits against the per-layer kernels, prompt 200 tokens (4 attention splits)."""
    from jax_llama_amd.config import get_preset
    cfg = get_preset("llama3-8b", num_hidden_layers=2, max_seq_len=512)
    model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).init_random(seed=3)
    monkeypatch.setattr(ops, "DECODE_MK", True)
    assert ops.decode_mk_ok(model, batch, 1, None)
    g = torch.Generator().manual_seed(5)
    toks = torch.randint(0, cfg.vocab_size, (batch, 200), generator=g, dtype=torch.int32)
    mask = torch.ones_like(toks)
    lm, hm, km, nxt = _decode_once(model, toks, mask, True, monkeypatch)
    assert ops.decode_mk_error(DEV) == 0
    ll, hl, kl, _ = _decode_once(model, toks, mask, False, monkeypatch)
    assert rel_err(hm, hl) < 1e-2, rel_err(hm, hl)
    assert rel_err(lm, ll) < 2e-2, rel_err(lm, ll)
    assert rel_err(km, kl) < 1e-2
