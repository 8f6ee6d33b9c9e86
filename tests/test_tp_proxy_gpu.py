"""The one-GPU tensor-parallel rank proxy (``parallel.TPRankProxyComm``, ``bench.py`` ``tp_rank_proxy``): rank 0's
shards of a Llama-3-70B MP8 model with every per-token collective on a world-1 instance of the custom kernels.

  * decode runs under hipGraph replay with the row-parallel GEMVs exchanging their partials themselves
    (``csrc/kernels/gemv.hip`` MODE_TPRESID) -- greedy tokens bit-identical to the standalone collective kernels
    (one pinned GEMV variant for both: the same K order) and to eager decode;
  * the proxy decode-step latency harness returns sane numbers at B = 1 and 32.
Reference: README.md:52-53 (70B needs MP = 8); partition.py:67,70 (the row-parallel all-reduces)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def proxy_model():
    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel import TPRankProxyComm
    cfg = get_preset("llama3-70b", max_seq_len=256, num_hidden_layers=2)
    comm = TPRankProxyComm.create(8, fused_hidden=cfg.hidden_size)
    assert comm.fused is not None
    model = LLaMAForCausalLM(cfg, device="cuda", comm=comm, _do_init=False).init_random(seed=11)
    yield cfg, comm, model
    del model
    comm.close()
    torch.cuda.empty_cache()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("variant", [1, 16, 26])
def test_proxy_fused_row_parallel_matches_standalone(proxy_model, variant):
    """variant 16: the split-K GEMV (2 workgroups per column group; only the last arriver exchanges); 26: 4 tiles x 8 waves
    per workgroup on packed x, K over 4 workgroups."""
    from jax_llama_amd import ops
    from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
    cfg, comm, model = proxy_model
    toks = torch.randint(3, cfg.vocab_size, (4, 12), generator=torch.Generator().manual_seed(2), dtype=torch.int32)
    gc = GenerationConfig(max_length=12 + 12, do_sample=False, pad_token_id=0, eos_token_id=-1)

    def greedy(use_graph):
        e = DecodeEngine(model, toks.shape[0], gc.max_length, use_graph=use_graph)
        out = e.run(toks, None, gc).cpu().clone()
        del e
        return out

    assert comm.fused.can_fuse(toks.shape[0], cfg.hidden_size)
    saved = ops.GEMV_VARIANT
    ops.GEMV_VARIANT = variant
    try:
        fused_graph = greedy(True)
        fused_eager = greedy(False)
        f, comm.fused = comm.fused, None
        try:
            standalone = greedy(True)
        finally:
            comm.fused = f
    finally:
        ops.GEMV_VARIANT = saved
    assert torch.equal(fused_graph, fused_eager)
    assert torch.equal(fused_graph, standalone)
    assert comm.fused.error() == 0 and comm.custom.error() == 0
    comm.check()


@pytest.mark.timeout(240)
def test_proxy_decode_latency(proxy_model):
    from jax_llama_amd.runtime.benchmark import decode_latency
    cfg, comm, model = proxy_model
    for b in (1, 32):
        r = decode_latency(model, b, prompt_len=32, gen_len=48, steps=16)
        assert 0 < r["decode_ms_per_token"] < 50, r
    comm.check()
