"""Native (deployed-form) safetensors checkpoint: save_pretrained / from_pretrained round trip.

The reference has no save path; this is the framework's resume format.
CPU: exact weights and identical logits after reload, a TP-degree mismatch is rejected, and a
2-rank gloo TP model saves one file per rank that reloads into the same sharded model. GPU: the
reload lands in the MFMA-packed layout bit-for-bit.
"""
from __future__ import annotations

import os

import pytest
import torch
import torch.multiprocessing as mp

from helpers import build, gpu_config, tiny_config
from test_distributed_cpu import _free_port


def _same_weights(a, b):
    assert torch.equal(a.wte.cpu(), b.wte.cpu()) and torch.equal(a.ln_f.cpu(), b.ln_f.cpu())
    assert torch.equal(a.lm_head.dense().cpu(), b.lm_head.dense().cpu())
    for la, lb in zip(a.layers, b.layers):
        for name in ("qkv", "o", "gu", "down"):
            assert torch.equal(getattr(la, name).dense().cpu(), getattr(lb, name).dense().cpu()), name
        assert torch.equal(la.attention_norm.cpu(), lb.attention_norm.cpu())


def test_save_and_reload_cpu(tmp_path):
    from jax_llama_amd.models import LLaMAForCausalLM
    cfg = tiny_config()
    model, _, _, _ = build(cfg, seed=5)
    model.save_pretrained(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["config.json", "jla_native.json", "model-rank00-of-01.safetensors"]
    again = LLaMAForCausalLM.from_pretrained(str(tmp_path))
    assert again.config == cfg
    _same_weights(model, again)
    toks = torch.randint(3, cfg.vocab_size, (2, 7), dtype=torch.int32)
    assert torch.equal(model(toks).logits, again(toks).logits)


def test_tp_mismatch_is_rejected(tmp_path):
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel.comm import TPComm
    model, _, _, _ = build(tiny_config(), seed=5)
    model.save_pretrained(str(tmp_path))
    with pytest.raises(ValueError, match="tp=1"):
        LLaMAForCausalLM.from_pretrained(str(tmp_path), comm=TPComm(size=2, rank=0))


def _tp_worker(rank, world, port, path, toks, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import torch.distributed as dist

        from jax_llama_amd.models import LLaMAForCausalLM
        from jax_llama_amd.parallel import TPComm, init_distributed
        ctx = init_distributed(backend="gloo", device_type="cpu")
        ctx.setup_mesh(tp=world)
        comm = TPComm.from_context(ctx)
        cfg = tiny_config(intermediate_size=128)
        _, _, _, params = build(cfg, seed=9)
        model = LLaMAForCausalLM(cfg, comm=comm, _do_init=False).load_params(params)
        model.save_pretrained(path)
        dist.barrier()
        again = LLaMAForCausalLM.from_pretrained(path, comm=comm)
        a, b = model(toks).logits, again(toks).logits
        if rank == 0:
            q.put(("ok", bool(torch.equal(a, b)), sorted(os.listdir(path))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc(), None))


def test_tp2_save_reload_gloo(tmp_path):
    toks = torch.randint(3, 256, (2, 6), dtype=torch.int32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, str(tmp_path), toks, q)) for r in range(2)]
    for p in procs:
        p.start()
    status, same, files = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", same
    assert same
    assert "model-rank00-of-02.safetensors" in files and "model-rank01-of-02.safetensors" in files


@pytest.mark.gpu
def test_save_reload_gpu_packed_exact(tmp_path):
    from jax_llama_amd.models import LLaMAForCausalLM
    cfg = gpu_config()
    model, _, _, _ = build(cfg, device="cuda", seed=3)
    model.save_pretrained(str(tmp_path))
    again = LLaMAForCausalLM.from_pretrained(str(tmp_path), device="cuda")
    for la, lb in zip(model.layers, again.layers):
        assert torch.equal(la.qkv.weight, lb.qkv.weight) and torch.equal(la.gu.weight, lb.gu.weight)
    toks = torch.randint(3, cfg.vocab_size, (2, 9), dtype=torch.int32)
    assert torch.equal(model(toks).logits, again(toks).logits)
