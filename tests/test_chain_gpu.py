"""Decode chain (``csrc/kernels/chain.hip``): wo -> w1|w3 -> w2 -> next layer's wqkv in ONE launch at M <= 16,
with in-launch agent-scope hand-offs. Checked against the unchained per-op path (the decode GEMV pinned to the
variant whose tiling and summation order the chain stages use -> bit-identical), against the CPU path, under
hipGraph replay, and at Llama-3-8B layer dimensions (the hand-off fan-in of 256 / 896 / 192-workgroup stages)."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd import LLaMAConfig, ops
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
from helpers import build, gpu_config, left_padded_batch, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _forward(model, toks, chain: bool):
    saved_c, saved_v = ops.DECODE_CHAIN, ops.GEMV_VARIANT
    ops.DECODE_CHAIN, ops.GEMV_VARIANT = chain, 1
    try:
        return model(toks).logits.cpu()
    finally:
        ops.DECODE_CHAIN, ops.GEMV_VARIANT = saved_c, saved_v


@pytest.mark.parametrize("kv_heads,shape", [(1, (1, 1)), (2, (3, 5)), (1, (16, 1)), (2, (2, 8))])
def test_chain_matches_unchained_toy(kv_heads, shape):
    cfg = gpu_config(num_attention_heads=2, num_key_value_heads=kv_heads)
    cpu, _, _, params = build(cfg, seed=1)
    gpu = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks = torch.randint(0, cfg.vocab_size, shape, dtype=torch.int32)
    a = _forward(gpu, toks, True)
    b = _forward(gpu, toks, False)
    assert torch.equal(a, b)
    assert rel_err(a, cpu(toks).logits) < 2e-2
    gpu.chain_state().check()
    assert int(gpu.chain_state().epoch[0].item()) >= 1


@pytest.mark.parametrize("m", [1, 8, 16])
def test_chain_llama3_8b_layer_dims(m):
    """Two layers at Llama-3-8B dimensions (D 4096, F 14336, 32 / 8 heads): stage grids of 256, 896, 256 and 192
    workgroups, i.e. the real fan-in of every hand-off."""
    cfg = LLaMAConfig(vocab_size=512, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
                      num_attention_heads=32, num_key_value_heads=8, max_sequence_length=64, rms_norm_eps=1e-5)
    model = LLaMAForCausalLM(cfg, device=DEV, seed=3)
    toks = torch.randint(0, cfg.vocab_size, (m, 1), dtype=torch.int32)
    a = _forward(model, toks, True)
    b = _forward(model, toks, False)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    model.chain_state().check()


def test_chain_graph_replay_and_generation():
    """Greedy generation at batch 2 (chained decode steps, hipGraph replay) == eager unchained generation."""
    cfg = gpu_config()
    _, _, _, params = build(cfg, seed=5)
    gpu = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks, mask = left_padded_batch([5, 8], 8, cfg.vocab_size, pad=2, seed=6)
    gc = GenerationConfig(max_length=48, do_sample=False, pad_token_id=2, eos_token_id=2)
    saved = ops.DECODE_CHAIN, ops.GEMV_VARIANT
    ops.DECODE_CHAIN, ops.GEMV_VARIANT = True, 1
    try:
        a = DecodeEngine(gpu, 2, 48, use_graph=True).run(toks, mask, gc).clone()
        ops.DECODE_CHAIN = False
        b = DecodeEngine(gpu, 2, 48, use_graph=False).run(toks, mask, gc).clone()
    finally:
        ops.DECODE_CHAIN, ops.GEMV_VARIANT = saved
    assert torch.equal(a, b)
    gpu.chain_state().check()
