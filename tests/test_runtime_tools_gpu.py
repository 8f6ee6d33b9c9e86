"""Runtime tooling on the device: the decode-step launch count read from the captured hipGraph (bench.py reports it),
and CU-masked streams with the workgroup-placement census (csrc/kernels/placement.hip; the round-6 CU-partition
measurements, profiles/README.md)."""
from __future__ import annotations

import pytest
import torch

from helpers import gpu_config
from jax_llama_amd import ops
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.benchmark import decode_latency

pytestmark = pytest.mark.gpu


def test_decode_kernels_counted_from_graph():
    cfg = gpu_config(num_hidden_layers=3)
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=3)
    p = decode_latency(model, 4, prompt_len=8, gen_len=8)
    n = p["kernels_per_step"]
    # every layer launches at least its qkv, o, gate_up and down projections; plus embedding / lm_head / update
    assert n >= 4 * cfg.num_hidden_layers + 2, p
    assert p["kernels_per_layer"] == round(n / cfg.num_hidden_layers, 2)


def _census(e, stream, blocks=2048):
    out = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(stream):
        e.cu_census(out)
    torch.cuda.synchronize()
    cus = set()
    for hw, xcc in out.view(-1, 2).cpu().tolist():
        hw &= 0xFFFFFFFF
        cus.add((xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF))
    return cus


def test_cu_masked_stream_places_workgroups_on_its_cus():
    e = ops.ext()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    everywhere = _census(e, torch.cuda.current_stream())
    assert len(everywhere) == ncu
    k = ncu // 4
    words = [0] * ((ncu + 31) // 32)
    for b in range(k):
        words[b // 32] |= 1 << (b % 32)
    raw = e.cu_mask_stream(words)
    try:
        assert e.cu_mask_of(raw, len(words)) == words
        s = torch.cuda.ExternalStream(raw)
        placed = _census(e, s)
        assert len(placed) == k and placed <= everywhere
    finally:
        torch.cuda.synchronize()
        e.stream_destroy(raw)
