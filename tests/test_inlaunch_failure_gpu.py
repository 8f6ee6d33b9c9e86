"""Failure detection of the in-launch waits (SURVEY §5 failure detection; the reference has none:
/root/reference/jax_llama/generation.py:28-41 just runs).

The fused small-batch qkv + attention launch (csrc/kernels/gemv.hip qkv_attn_kernel) makes its attention workgroups
wait for the qkv workgroups' publish, bounded by a timeout that sets an error word. With the diagnostic knob the qkv
workgroups never publish: the engine must raise instead of returning tokens, refuse the fused path afterwards, and
produce the same tokens as before through the two-kernel path."""
from __future__ import annotations

import pytest
import torch

from helpers import gpu_config
from jax_llama_amd import ops
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.engine import GenerationConfig

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused_o", [0, 1])
def test_qkv_attn_timeout_raises_and_recovers(fused_o):
    """(fused_o: the launch also runs the o projection, whose workgroups then see the attention side's error word and
    leave the residual alone.)"""
    e = ops.ext()
    # 8 query heads per kv head, B = 1: the shape the fused launch serves (the 70B tensor-parallel shard)
    cfg = gpu_config(hidden_size=1024, intermediate_size=512, num_attention_heads=8, num_key_value_heads=1,
                     vocab_size=512, num_hidden_layers=2)
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=5)
    ids = torch.randint(3, cfg.vocab_size, (1, 12), dtype=torch.int32)
    gc = GenerationConfig(max_length=40, do_sample=False, pad_token_id=0, eos_token_id=-1)
    saved, saved_o = ops.QKV_ATTN, ops.QKV_ATTN_O
    ops.QKV_ATTN_O = fused_o
    try:
        x = torch.zeros(1, cfg.hidden_size, dtype=torch.bfloat16, device="cuda")
        cache = model.init_cache(1, 40)
        assert ops.qkv_attention_splits(x, model.layers[0].qkv, cache.layer(0)[0], 1, 8, 1) > 0, "fused path not used"
        assert not fused_o or ops.qkv_attention_o_groups(x, model.layers[0].o, 8, 1) > 0, "fused o not used"
        del cache
        ops.QKV_ATTN = 0
        two = model.generate(ids, generation_config=gc).sequences.cpu()  # the two-kernel path
        ops.QKV_ATTN = saved
        model.generate(ids, generation_config=gc)  # fused, healthy
        e.qkv_attn_set_diag(1)
        with pytest.raises(ops.InLaunchTimeout):
            model.generate(ids, generation_config=gc)
        e.qkv_attn_set_diag(0)
        assert ops.QKV_ATTN == 0, "the fused path must be refused after a timeout"
        again = model.generate(ids, generation_config=gc).sequences.cpu()
        assert torch.equal(two, again), "after the failure: the two-kernel path's tokens"
        ops.check_inlaunch()  # the words were re-zeroed: nothing left to report
    finally:
        e.qkv_attn_set_diag(0)
        ops.QKV_ATTN = saved
        ops.QKV_ATTN_O = saved_o
