"""Whole-model parity on the MI355X: HIP-kernel model vs the CPU execution path (same bf16 rounding
points) and vs the independent fp32 oracle; hipGraph-replayed decode vs eager decode."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
from helpers import build, gpu_config, left_padded_batch, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(cfg, seed=0):
    model_cpu, oracle, sd, params = build(cfg, seed=seed)
    model_gpu = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    return model_cpu, model_gpu, oracle


@pytest.mark.parametrize("kv_heads", [2, 1])
def test_logits_gpu_vs_cpu_and_oracle(kv_heads):
    cfg = gpu_config(num_attention_heads=2, num_key_value_heads=kv_heads)
    cpu, gpu, oracle = _pair(cfg)
    toks = torch.randint(0, cfg.vocab_size, (3, 20), dtype=torch.int32)
    lg = gpu(toks).logits.cpu()
    lc = cpu(toks).logits
    lo = oracle.forward(toks)
    assert rel_err(lg, lc) < 2e-2
    assert rel_err(lg, lo) < 5e-2


def test_padded_prefill_then_decode_gpu():
    cfg = gpu_config()
    cpu, gpu, oracle = _pair(cfg, seed=2)
    toks, mask = left_padded_batch([3, 9, 12], 12, cfg.vocab_size, pad=2)
    pos = mask.cumsum(-1) - 1
    lg = gpu(toks, attention_mask=mask, position_ids=pos).logits.cpu()
    lo = oracle.forward(toks, mask, pos)
    m = mask.bool()
    assert rel_err(lg[m], lo[m]) < 5e-2
    assert torch.isfinite(lg).all()


@pytest.mark.parametrize("batch", [1, 4, 20])
def test_greedy_generation_gpu_matches_cpu_path(batch):
    cfg = gpu_config()
    cpu, gpu, oracle = _pair(cfg, seed=3)
    lens = [max(2, 11 - (3 * i) % 9) for i in range(batch)]
    toks, mask = left_padded_batch(lens, 11, cfg.vocab_size, pad=2, seed=4)
    gc = dict(max_length=40, do_sample=False, pad_token_id=2, eos_token_id=2)
    got = gpu.generate(toks, attention_mask=mask, generation_config=GenerationConfig(**gc)).sequences.cpu()
    want = cpu.generate(toks, attention_mask=mask, generation_config=GenerationConfig(**gc)).sequences
    # identical bf16 rounding points -> identical greedy tokens except after exact near-ties
    agree = (got.long() == want.long()).float().mean().item()
    assert agree > 0.97, agree
    assert torch.equal(got[:, :11], toks)


def test_graph_replay_matches_eager():
    cfg = gpu_config()
    _, gpu, _ = _pair(cfg, seed=5)
    toks, mask = left_padded_batch([5, 8], 8, cfg.vocab_size, pad=2, seed=6)
    gc = GenerationConfig(max_length=48, do_sample=False, pad_token_id=2, eos_token_id=2)
    e1 = DecodeEngine(gpu, 2, 48, use_graph=True)
    a = e1.run(toks, mask, gc).clone()
    e2 = DecodeEngine(gpu, 2, 48, use_graph=False)
    b = e2.run(toks, mask, gc).clone()
    assert torch.equal(a, b)


def test_sampling_gpu_seeded():
    cfg = gpu_config()
    _, gpu, _ = _pair(cfg, seed=7)
    toks, mask = left_padded_batch([4, 6], 6, cfg.vocab_size, pad=2, seed=8)
    gc = dict(max_length=30, do_sample=True, temperature=0.8, top_p=0.95, pad_token_id=2, eos_token_id=2)
    a = gpu.generate(toks, mask, GenerationConfig(seed=11, **gc)).sequences.cpu()
    b = gpu.generate(toks, mask, GenerationConfig(seed=11, **gc)).sequences.cpu()
    assert torch.equal(a, b)
    assert int(a.min()) >= 0 and int(a.max()) < cfg.vocab_size


def test_random_init_8b_shapes_one_layer():
    """Synthetic path of bench.py at the real Llama-3-8B layer shapes (1 layer to keep it fast)."""
    from jax_llama_amd.config import get_preset
    cfg = get_preset("llama3-8b", num_hidden_layers=1)
    m = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).init_random(seed=0)
    toks = torch.randint(0, cfg.vocab_size, (2, 16), dtype=torch.int32)
    gc = GenerationConfig(max_length=24, do_sample=False, pad_token_id=0, eos_token_id=-1)
    seq = m.generate(toks, generation_config=gc).sequences
    assert seq.shape == (2, 24)
    assert int(seq.min()) >= 0 and int(seq.max()) < cfg.vocab_size


def test_graph_recaptured_after_workspace_growth():
    """a cached decode graph must not replay with freed workspace buffers. Run,
    run a longer prompt on ANOTHER engine (grows the shared workspaces), run the first engine again:
    every run must equal an eager run."""
    from jax_llama_amd import ops
    ops.workspace.clear()  # earlier tests may already have grown the shared buffers past this test's sizes
    cfg = gpu_config()
    _, gpu, _ = _pair(cfg, seed=12)
    gc = GenerationConfig(max_length=40, do_sample=False, pad_token_id=2, eos_token_id=-1)
    toks, mask = left_padded_batch([4, 7], 8, cfg.vocab_size, pad=2, seed=13)
    e1 = DecodeEngine(gpu, 2, 40, use_graph=True)
    first = e1.run(toks, mask, gc).clone()
    gen0 = ops.workspace.generation
    big, bmask = left_padded_batch([30] * 24, 30, cfg.vocab_size, pad=2, seed=14)
    DecodeEngine(gpu, 24, 40, use_graph=True).run(big, bmask, gc)
    assert ops.workspace.generation > gen0  # the larger batch reallocated shared scratch
    again = e1.run(toks, mask, gc).clone()
    eager = DecodeEngine(gpu, 2, 40, use_graph=False).run(toks, mask, gc).clone()
    assert torch.equal(first, eager) and torch.equal(again, eager)


@pytest.mark.parametrize("path", ["gemv", "tiled"])
def test_fused_argmax_engine_path(monkeypatch, path):
    """the lm_head with the argmax in its epilogue -- the decode GEMV's (M <= 64) or
    the tiled GEMM's (forced at small M) -- inside the captured decode step gives the same greedy
    sequences as logits + argmax."""
    from jax_llama_amd import ops
    from jax_llama_amd.runtime import engine as eng_mod
    cfg = gpu_config()
    cpu, gpu, _ = _pair(cfg, seed=15)
    toks, mask = left_padded_batch([6, 9, 9], 9, cfg.vocab_size, pad=2, seed=16)
    gc = GenerationConfig(max_length=30, do_sample=False, pad_token_id=2, eos_token_id=-1)
    monkeypatch.setattr(ops, "ARGMAX_FUSED_MIN_M", 1)
    monkeypatch.setattr(ops, "SKINNY_ARGMAX", path == "gemv")
    fused = DecodeEngine(gpu, 3, 30, use_graph=True).run(toks, mask, gc).clone()
    monkeypatch.setattr(eng_mod, "FUSED_GREEDY", False)
    plain = DecodeEngine(gpu, 3, 30, use_graph=True).run(toks, mask, gc).clone()
    assert torch.equal(fused, plain)


def test_precision_highest_logits():
    """precision='highest' (jax_test.py:433): fp32 lm_head weights + fp32 GEMM; closer to the fp32
    oracle than the default bf16 lm_head."""
    cfg = gpu_config()
    _, oracle, _, params = build(cfg, seed=17)
    hi = LLaMAForCausalLM(cfg, device=DEV, _do_init=False, precision="highest").load_params(params)
    lo = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).load_params(params)
    toks = torch.randint(3, cfg.vocab_size, (2, 10), dtype=torch.int32)
    want = oracle.forward(toks)
    e_hi = rel_err(hi(toks).logits.cpu(), want)
    e_lo = rel_err(lo(toks).logits.cpu(), want)
    assert e_hi < 5e-2 and e_hi <= e_lo * 1.05, (e_hi, e_lo)
    gc = GenerationConfig(max_length=16, do_sample=False, pad_token_id=0, eos_token_id=-1)
    seq = hi.generate(toks, generation_config=gc).sequences
    assert seq.shape == (2, 16)


def test_benchmark_helpers_at_max_sequence_length():
    """bench.py's extra points (runtime/benchmark.py): TTFT at a prompt as long as max_sequence_length (the
    RoPE table covers 2x) and one decode latency point, on a small random model."""
    from jax_llama_amd.runtime.benchmark import decode_latency, time_to_first_token
    cfg = gpu_config(max_sequence_length=64)
    m = LLaMAForCausalLM(cfg, device="cuda", seed=0)
    t = time_to_first_token(m, 1, cfg.max_sequence_length, reps=2)
    assert t["ttft_ms"] > 0 and t["prompt_len"] == cfg.max_sequence_length
    d = decode_latency(m, 2, prompt_len=8, gen_len=16, steps=4)
    assert d["decode_ms_per_token"] > 0


@pytest.mark.parametrize("rows", [12, 20, 32])
def test_packed_activations_decode_rows(rows):
    """Decode-shaped forward (one token per row) with the packed activation copies (ops.PACKED_X) vs without:
    same logits up to the GEMV variants' summation order, and vs the CPU path."""
    from jax_llama_amd import ops
    cfg = gpu_config(num_attention_heads=2, num_key_value_heads=1)
    cpu, gpu, _ = _pair(cfg, seed=9)
    toks = torch.randint(0, cfg.vocab_size, (rows, 1), dtype=torch.int32)
    saved = ops.PACKED_X
    try:
        ops.PACKED_X = True
        a = gpu(toks).logits.cpu()
        ops.PACKED_X = False
        b = gpu(toks).logits.cpu()
    finally:
        ops.PACKED_X = saved
    assert rel_err(a, b) < 1e-2
    assert rel_err(a, cpu(toks).logits) < 2e-2


def test_output_attentions_gpu_same_logits_and_causal_weights():
    """output_attentions on the GPU: the layer outputs still come from the attention kernel (logits identical to the
    run without the flag), and the returned weights are the causal softmax rows (reference model.py:277-286)."""
    cfg = gpu_config(num_hidden_layers=2)
    _, gpu, _ = _pair(cfg, seed=4)
    toks = torch.randint(0, cfg.vocab_size, (2, 9), dtype=torch.int32)
    plain = gpu(toks).logits.float().cpu()
    out = gpu(toks, output_attentions=True)
    assert torch.equal(out.logits.float().cpu(), plain)
    assert len(out.attentions) == cfg.num_hidden_layers
    w = out.attentions[0].float().cpu()
    assert w.shape == (2, cfg.num_attention_heads, 9, 9)
    assert torch.allclose(w.sum(-1), torch.ones_like(w.sum(-1)), atol=1e-4)
    assert torch.all(torch.triu(w[0, 0], 1) == 0)


def test_decode_fused_o_projection_matches_two_launches():
    """Greedy decode with the Llama-3-70B tensor-parallel shard's attention geometry (8 query heads per kv head,
    H * Dh = 1024) and the o projection inside the fused qkv + attention launch (ops.QKV_ATTN_O) produces exactly the
    tokens of the two-launch step with the standalone GEMV of the same geometry (variant 6: 2 tiles x 4 waves; the two
    are bit-identical, tests/test_kernels_gpu.py test_qkv_attention_fused_o_projection), graph-captured decode."""
    from jax_llama_amd import ops
    cfg = gpu_config(hidden_size=1024, intermediate_size=512, num_attention_heads=8, num_key_value_heads=1,
                     vocab_size=512, num_hidden_layers=2)
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=11)
    ids = torch.randint(3, cfg.vocab_size, (1, 12), dtype=torch.int32)
    gc = GenerationConfig(max_length=48, do_sample=False, pad_token_id=0, eos_token_id=-1)
    x = torch.zeros(1, cfg.hidden_size, dtype=torch.bfloat16, device="cuda")
    saved_v, saved_o = ops.GEMV_VARIANT, ops.QKV_ATTN_O
    try:
        ops.GEMV_VARIANT = 6
        out = {}
        for fo in (0, 1):
            ops.QKV_ATTN_O = fo
            assert ops.qkv_attention_o_groups(x, model.layers[0].o, 8, 1) == (1024 // 32 if fo else 0)
            out[fo] = model.generate(ids, generation_config=gc).sequences.cpu()
    finally:
        ops.GEMV_VARIANT, ops.QKV_ATTN_O = saved_v, saved_o
    assert torch.equal(out[0], out[1])
