"""Model vs the independent fp32 oracle on the CPU execution path (reference ops).

Mirrors jax_test.py's unit/integration parity ladder (RMSNorm, RoPE, attention, block,
full transformer logits, greedy generations) at the tiny fixture dims.
"""
import math

import pytest
import torch

from jax_llama_amd.ops import reference as ref
from helpers import build, left_padded_batch, rel_err, tiny_config
from oracle import apply_rotary_emb, precompute_freqs_cis


def test_rope_matches_complex_oracle():
    dh, s = 16, 40
    table = ref.rope_table(dh, 128, 10000.0)
    x = torch.randn(2, s, 3, dh)
    pos = torch.arange(s).expand(2, s)
    fc = precompute_freqs_cis(dh, 128)[pos]
    want = apply_rotary_emb(x, fc)
    got = ref.apply_rope(x.reshape(-1, 3, dh), table, pos.reshape(-1)).reshape(2, s, 3, dh)
    assert (got - want).abs().max() < 1e-5


def test_scaled_rope_changes_low_freqs_only():
    a = ref.rope_table(128, 16, 500000.0)
    b = ref.rope_table(128, 16, 500000.0, scaled=True)
    assert torch.allclose(a[:, :8], b[:, :8])
    assert not torch.allclose(a[:, -8:], b[:, -8:])


def test_rmsnorm_reference():
    x = torch.randn(4, 64)
    w = torch.randn(64)
    got = ref.rmsnorm(x, w, 1e-5)
    want = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w
    assert (got - want).abs().max() < 1e-6


@pytest.mark.parametrize("kv_heads", [4, 2, 1])
def test_full_model_logits_vs_oracle(kv_heads):
    cfg = tiny_config(num_key_value_heads=kv_heads)
    model, oracle, *_ = build(cfg)
    toks = torch.randint(0, cfg.vocab_size, (2, 12), dtype=torch.int32)
    got = model(toks).logits
    want = oracle.forward(toks)
    assert got.shape == (2, 12, cfg.vocab_size)
    assert rel_err(got, want) < 3e-2


def test_padded_batch_logits_vs_oracle():
    cfg = tiny_config()
    model, oracle, *_ = build(cfg)
    toks, mask = left_padded_batch([5, 9, 12], 12, cfg.vocab_size, pad=2)
    pos = (mask.cumsum(-1) - 1)
    got = model(toks, attention_mask=mask, position_ids=pos).logits
    want = oracle.forward(toks, mask, pos)
    # compare valid (non-pad) positions only
    m = mask.bool()
    assert rel_err(got[m], want[m]) < 3e-2


def test_incremental_cache_matches_full_forward():
    cfg = tiny_config()
    model, oracle, *_ = build(cfg)
    toks = torch.randint(0, cfg.vocab_size, (2, 10), dtype=torch.int32)
    full = model(toks).logits
    kw = model.prepare_inputs_for_generation(toks[:, :6], max_length=10)
    out = model(toks[:, :6], attention_mask=kw["attention_mask"], position_ids=kw["position_ids"],
                past_key_values=kw["past_key_values"])
    assert rel_err(out.logits, full[:, :6]) < 1e-5
    kw = model.update_inputs_for_generation(out, kw)
    for t in range(6, 10):
        out = model(toks[:, t:t + 1], attention_mask=kw["attention_mask"], position_ids=kw["position_ids"],
                    past_key_values=kw["past_key_values"])
        assert rel_err(out.logits[:, 0], full[:, t]) < 2e-2
        kw = model.update_inputs_for_generation(out, kw)


def test_hidden_states_and_attentions_outputs():
    cfg = tiny_config()
    model, *_ = build(cfg)
    toks = torch.randint(0, cfg.vocab_size, (1, 7), dtype=torch.int32)
    out = model(toks, output_hidden_states=True, output_attentions=True)
    assert len(out.hidden_states) == cfg.num_hidden_layers + 1
    assert len(out.attentions) == cfg.num_hidden_layers
    w = out.attentions[0]
    assert w.shape == (1, cfg.num_attention_heads, 7, 7)
    assert torch.allclose(w.sum(-1), torch.ones_like(w.sum(-1)), atol=1e-5)
    assert torch.all(torch.triu(w[0, 0], 1) == 0)


def test_greedy_generation_matches_oracle():
    cfg = tiny_config(num_hidden_layers=2)
    model, oracle, *_ = build(cfg, seed=3)
    toks, mask = left_padded_batch([4, 7], 7, cfg.vocab_size, pad=2, seed=1)
    from jax_llama_amd.runtime.engine import GenerationConfig
    gc = GenerationConfig(max_length=15, do_sample=False, pad_token_id=2, eos_token_id=2)
    got = model.generate(toks, attention_mask=mask, generation_config=gc).sequences
    want = oracle.greedy(toks.long(), mask.long(), 15, pad=2, eos=2)
    # bf16 model vs fp32 oracle: allow divergence only after a near-tie; here require equality
    assert torch.equal(got.long(), want)


@pytest.mark.parametrize("do_sample", [False, True])
def test_prefill_row_chunks_match_one_forward(do_sample, monkeypatch):
    """The engine's prefill in row chunks (large batches: at most PREFILL_TOKENS prompt tokens per forward, each chunk
    writing its own rows of the KV cache) generates exactly what one whole-batch prefill does, padding mask included."""
    from jax_llama_amd.runtime import engine
    from jax_llama_amd.runtime.engine import GenerationConfig
    cfg = tiny_config(num_hidden_layers=2)
    model, *_ = build(cfg, seed=4)
    toks, mask = left_padded_batch([4, 7, 2, 7, 5], 7, cfg.vocab_size, pad=2, seed=3)
    gc = GenerationConfig(max_length=14, do_sample=do_sample, temperature=0.8, top_p=0.95, pad_token_id=2,
                          eos_token_id=-1, seed=11)
    whole = model.generate(toks, attention_mask=mask, generation_config=gc).sequences.clone()
    engine._ENGINES.clear()
    monkeypatch.setattr(engine, "PREFILL_TOKENS", 14)  # 2 rows per forward: chunks of 2, 2, 1
    chunked = model.generate(toks, attention_mask=mask, generation_config=gc).sequences
    engine._ENGINES.clear()
    assert torch.equal(whole, chunked)


def test_sampling_is_seeded_and_valid():
    cfg = tiny_config(num_hidden_layers=2)
    model, *_ = build(cfg, seed=5)
    toks, mask = left_padded_batch([3, 5], 5, cfg.vocab_size, pad=2)
    from jax_llama_amd.runtime.engine import GenerationConfig
    gc = dict(max_length=12, do_sample=True, temperature=0.8, top_p=0.95, pad_token_id=2, eos_token_id=2)
    a = model.generate(toks, mask, GenerationConfig(seed=7, **gc)).sequences
    b = model.generate(toks, mask, GenerationConfig(seed=7, **gc)).sequences
    assert torch.equal(a, b)
    assert a.shape == (2, 12)
    assert torch.equal(a[:, :5], toks)
    assert int(a.min()) >= 0 and int(a.max()) < cfg.vocab_size


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors (the sampler's RNG, bit-exact with the kernel)."""
    import numpy as np
    from jax_llama_amd.ops.reference import philox4x32_10
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = philox4x32_10(np.array([ctr], dtype=np.uint32), key)[0]
        assert tuple(int(x) for x in got) == want


def test_reference_sampler_semantics():
    from jax_llama_amd.ops import reference as ref
    torch.manual_seed(0)
    logits = torch.randn(64, 1000) * 3
    # top_k = 1 and tiny top_p are greedy
    assert torch.equal(ref.topk_sample(logits, 1, 1.0, 1.0, 5, 3), ref.argmax(logits))
    assert torch.equal(ref.topk_sample(logits, 50, 1.0, 1e-6, 5, 3), ref.argmax(logits))
    # sampled tokens lie in the top-k set, and change with the step / seed
    a = ref.topk_sample(logits, 10, 0.7, 0.9, 5, 3)
    top10 = logits.topk(10, -1).indices
    assert bool((top10 == a[:, None].long()).any(-1).all())
    assert not torch.equal(a, ref.topk_sample(logits, 10, 0.7, 0.9, 5, 4))
    assert not torch.equal(a, ref.topk_sample(logits, 10, 0.7, 0.9, 6, 3))
    # ties: lower index first
    v, i = ref.topk_sorted(torch.tensor([[1.0, 3.0, 3.0, 2.0, 3.0]]), 3)
    assert i.tolist() == [[1, 2, 4]]
    # frequencies follow softmax(top-k logits / T)
    row = torch.tensor([[2.0, 1.0, 0.5, 0.0, -1.0, -5.0]]).repeat(4000, 1)
    s = torch.cat([ref.topk_sample(row, 4, 1.0, 1.0, 1, st) for st in range(3)])
    freq = torch.bincount(s.long(), minlength=6).float() / s.numel()
    p = torch.softmax(row[0, :4], -1)
    assert freq[4:].sum() == 0
    assert (freq[:4] - p).abs().max() < 0.02


def test_llama2_7b_config_two_layer_greedy_plumbing():
    """BASELINE.json config 1: LLaMA-2 7B shapes (D 4096, 32 heads, F 11008, V 32000), 2 layers, random
    init, greedy decode at MP=1 through the reference ``LLaMA.generate`` surface (generation.py:22-45) --
    the jax_example.py plumbing on the CPU path. Checks the left-padded prompt, the EOS=pad convention and
    that each cached decode token is the argmax of a full (no-cache) forward over the sequence so far."""
    from types import SimpleNamespace

    from jax_llama_amd import LLaMA
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    cfg = get_preset("llama2-7b", num_hidden_layers=2)
    assert (cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size, cfg.num_attention_heads) == (4096, 11008, 32000, 32)
    model = LLaMAForCausalLM(cfg, device="cpu", _do_init=False).init_random(seed=0)
    tok = SimpleNamespace(eos_id=2, bos_id=1)
    gen = LLaMA(None, model, tok)
    g = torch.Generator().manual_seed(3)
    tokens = torch.full((2, 6), tok.eos_id, dtype=torch.int32)
    tokens[0] = torch.randint(3, cfg.vocab_size, (6,), generator=g)
    tokens[1, 2:] = torch.randint(3, cfg.vocab_size, (4,), generator=g)
    mask = (tokens != tok.eos_id).to(torch.int32)
    out = gen.generate(tokens, mask, max_gen_len=3, temperature=0.0)
    assert out.shape == (2, 9) and torch.equal(out[:, :6], tokens)
    assert torch.equal(out, gen.generate(tokens, mask, max_gen_len=3, temperature=0.0))
    for row in range(2):
        n0 = int(mask[row].sum())
        seq = out[row:row + 1, 6 - n0:]  # drop the left padding: positions restart at 0 either way
        logits = model(seq).logits[0]
        for j in range(3):
            step = logits[n0 - 1 + j]
            top2 = step.topk(2).values
            if float(top2[0] - top2[1]) > 1e-3 * float(step.abs().max()):  # skip near-ties (bf16 weights)
                assert int(step.argmax()) == int(seq[0, n0 + j]), (row, j)
