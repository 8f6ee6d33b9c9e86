"""Correctness at production shapes (reference jax_test.py:427-490 last-position logits at real checkpoint dims,
atol 1e-1; :492-522 32-token greedy equality).

  * Llama-3-8B real dims (D 4096, 32 q / 8 kv heads, F 14336, V 128256; 2 layers): the HIP model's logits against
    the independent fp32 oracle (tests/oracle.py) run in fp32 on the GPU, and its greedy tokens against the oracle's
    teacher-forced argmax;
  * the bench regime (bench.py: thousands of decode rows): at 768 rows the decode step runs the tiled GEMM plans,
    decode attention v4 (> 4096 (row, kv head) pairs) and the tiled GEMM with the argmax epilogue -- its greedy
    tokens against the same rows run at B = 8 through the decode GEMV path, both judged by the oracle's
    teacher-forced argmax gap (a near-tie broken differently costs at most the logits' rounding error)."""
from __future__ import annotations

import pytest
import torch

from helpers import argmax_gap, gpu_meta_state_dict, left_padded_batch, rel_err
from oracle import OracleLLaMA

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def llama3_8b_2l():
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.utils.checkpoint import meta_state_dict_to_params
    cfg = get_preset("llama3-8b", max_seq_len=256, num_hidden_layers=2)
    sd = gpu_meta_state_dict(cfg, seed=31)
    params = meta_state_dict_to_params(sd, cfg.num_hidden_layers)
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).load_params(params)
    oracle = OracleLLaMA(sd, cfg.num_hidden_layers, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.rms_norm_eps, cfg.rope_theta)
    del sd, params
    yield cfg, model, oracle
    del model, oracle
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
def test_llama3_8b_dims_logits_and_greedy_vs_fp32_oracle(llama3_8b_2l):
    from jax_llama_amd.runtime.engine import GenerationConfig
    cfg, model, oracle = llama3_8b_2l
    s = 48
    toks, mask = left_padded_batch([48, 31, 7, 40], s, cfg.vocab_size, pad=2, seed=5)
    pos = mask.cumsum(-1) - 1
    lg = model(toks, attention_mask=mask, position_ids=pos).logits
    lo = oracle.forward(toks, mask, pos)
    m = mask.bool().to(lg.device)
    assert torch.isfinite(lg).all()
    err_all = rel_err(lg[m], lo[m])
    err_last = rel_err(lg[:, -1], lo[:, -1])
    assert err_all < 5e-2, err_all
    assert err_last < 5e-2, err_last
    gc = GenerationConfig(max_length=s + 16, do_sample=False, pad_token_id=2, eos_token_id=-1)
    seq = model.generate(toks, attention_mask=mask, generation_config=gc).sequences.cpu()
    assert torch.equal(seq[:, :s], toks)
    gap = argmax_gap(oracle, seq, mask, s)
    assert gap < 1e-2, gap


@pytest.mark.timeout(600)
def test_bench_regime_greedy_matches_small_batch(llama3_8b_2l):
    from jax_llama_amd import ops
    from jax_llama_amd.runtime.benchmark import synthetic_prompts
    from jax_llama_amd.runtime.engine import GenerationConfig
    cfg, model, oracle = llama3_8b_2l
    b, s, gen = 768, 16, 8
    assert b * cfg.num_key_value_heads > 4096 and b >= ops.ARGMAX_FUSED_MIN_M  # v4 attention, tiled fused argmax
    prompts = synthetic_prompts(cfg.vocab_size, b, s, seed=12)
    gc = GenerationConfig(max_length=s + gen, do_sample=False, pad_token_id=0, eos_token_id=-1)
    big = model.generate(prompts, generation_config=gc).sequences.cpu()
    rows = [0, 1, 255, 256, 511, 512, 700, 767]
    small = model.generate(prompts[rows], generation_config=gc).sequences.cpu()
    ones = torch.ones(len(rows), s, dtype=torch.int32)
    gap_big = argmax_gap(oracle, big[rows], ones, s)
    gap_small = argmax_gap(oracle, small, ones, s)
    agree = (big[rows][:, s:] == small[:, s:]).float().mean().item()  # informative: a near-tie can flip a row
    assert gap_big < 1e-2, (gap_big, agree)
    assert gap_small < 1e-2, (gap_small, agree)
    assert agree > 0.5, agree
    assert int(big.min()) >= 0 and int(big.max()) < cfg.vocab_size


@pytest.mark.timeout(600)
def test_headline_regime_b4096_prompt128(llama3_8b_2l):
    """The exact benchmarked regime (bench.py: B = 4096, 128-token prompts): the prefill in two row chunks of
    M = 262,144 rows (tile-0 GEMMs, flash prefill; runtime/engine.py PREFILL_TOKENS) and the B = 4096 decode plans
    (tuned tiled GEMMs, v4 attention, the fused-argmax lm_head), 32 generated tokens; 8 rows spread over both chunks
    against the same rows run at B = 8, both judged by the fp32 oracle's teacher-forced argmax gap (reference
    jax_test.py:427-490, 492-522)."""
    from jax_llama_amd.runtime import engine
    from jax_llama_amd.runtime.benchmark import synthetic_prompts
    from jax_llama_amd.runtime.engine import GenerationConfig
    cfg, model, oracle = llama3_8b_2l
    b, s, gen = 4096, 128, 32
    assert b * s > engine.PREFILL_TOKENS  # the chunked prefill
    prompts = synthetic_prompts(cfg.vocab_size, b, s, seed=21)
    gc = GenerationConfig(max_length=s + gen, do_sample=False, pad_token_id=0, eos_token_id=-1)
    big = model.generate(prompts, generation_config=gc).sequences.cpu()
    engine._ENGINES.clear()
    torch.cuda.empty_cache()
    rows = [0, 1, 1023, 2047, 2048, 3000, 4000, 4095]
    small = model.generate(prompts[rows], generation_config=gc).sequences.cpu()
    ones = torch.ones(len(rows), s, dtype=torch.int32)
    gap_big = argmax_gap(oracle, big[rows], ones, s)
    gap_small = argmax_gap(oracle, small, ones, s)
    agree = (big[rows][:, s:] == small[:, s:]).float().mean().item()
    assert gap_big < 1e-2, (gap_big, agree)
    assert gap_small < 1e-2, (gap_small, agree)
    assert agree > 0.5, agree
    assert int(big.min()) >= 0 and int(big.max()) < cfg.vocab_size
