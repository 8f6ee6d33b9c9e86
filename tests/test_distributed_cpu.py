"""Tensor parallelism (explicit SPMD, partition.py rules) on CPU with the gloo backend.

Each rank holds its Megatron shard (column-parallel wq/wk/wv/w1/w3, row-parallel wo/w2 with an
all-reduce, vocab-parallel lm_head with an all-gather); outputs must match the single-process
model. Mirrors the reference's only multi-process path (jax_test.py:60-70, torchrun + NCCL), with
gloo standing in for RCCL so it runs without GPUs.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import build, left_padded_batch, tiny_config


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg_kw, toks, mask, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        from jax_llama_amd.models import LLaMAForCausalLM
        from jax_llama_amd.parallel import TPComm, init_distributed
        from jax_llama_amd.runtime.engine import GenerationConfig
        torch.manual_seed(0)
        ctx = init_distributed(backend="gloo", device_type="cpu")
        ctx.setup_mesh(tp=world)
        comm = TPComm.from_context(ctx)
        cfg = tiny_config(**cfg_kw)
        _, _, _, params = build(cfg, seed=11)
        model = LLaMAForCausalLM(cfg, comm=comm, _do_init=False).load_params(params)
        pos = mask.cumsum(-1) - 1
        logits = model(toks, attention_mask=mask, position_ids=pos).logits
        gc = GenerationConfig(max_length=toks.shape[1] + 6, do_sample=False, pad_token_id=2, eos_token_id=2)
        seq = model.generate(toks, attention_mask=mask, generation_config=gc).sequences
        gcs = GenerationConfig(max_length=toks.shape[1] + 6, do_sample=True, temperature=0.7, top_p=0.9,
                               pad_token_id=2, eos_token_id=2, seed=3)
        sseq = model.generate(toks, attention_mask=mask, generation_config=gcs).sequences
        if rank == 0:
            q.put(("ok", logits, seq, sseq))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced in the parent
        import traceback
        q.put(("err", traceback.format_exc(), None, None))


@pytest.mark.parametrize("world,kv", [(2, 2), (2, 4), (4, 4), (8, 8)])
def test_tensor_parallel_matches_single_process(world, kv):
    cfg_kw = dict(num_key_value_heads=kv, intermediate_size=128, vocab_size=256)
    if world == 8:  # 8 heads / 8 kv heads: one of each per rank (the 70B TP8 per-rank head layout has 1 kv head)
        cfg_kw.update(num_attention_heads=8, hidden_size=64)
    cfg = tiny_config(**cfg_kw)
    ref_model, _, _, _ = build(cfg, seed=11)
    toks, mask = left_padded_batch([5, 8], 8, cfg.vocab_size, pad=2, seed=2)
    pos = mask.cumsum(-1) - 1
    want = ref_model(toks, attention_mask=mask, position_ids=pos).logits
    from jax_llama_amd.runtime.engine import GenerationConfig
    want_seq = ref_model.generate(toks, attention_mask=mask, generation_config=GenerationConfig(
        max_length=14, do_sample=False, pad_token_id=2, eos_token_id=2)).sequences

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg_kw, toks, mask, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, logits, seq, sseq = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", logits
    m = mask.bool()
    assert (logits[m] - want[m]).abs().max() < 2e-2
    assert torch.equal(seq.long(), want_seq.long())
    assert sseq.shape == seq.shape and int(sseq.min()) >= 0 and int(sseq.max()) < cfg.vocab_size


def _tune_worker(rank, world, port, path, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), JLA_TUNE_FILE=path)
        from jax_llama_amd.ops import autotune
        from jax_llama_amd.parallel import TPComm, init_distributed
        ctx = init_distributed(backend="gloo", device_type="cpu")
        ctx.setup_mesh(tp=world)
        comm = TPComm.from_context(ctx)
        with autotune.tp_scope(comm):
            got = autotune._collective(lambda: (rank + 1, 10 * (rank + 1)))  # each rank would "measure" differently
        local = autotune._collective(lambda: rank)  # outside a TP scope: every process decides for itself
        dist.barrier()
        dist.destroy_process_group()
        q.put(("ok", rank, (got, local)))
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", rank, traceback.format_exc()))


def test_autotune_decisions_are_collective_under_tp(tmp_path):
    """Under TP every rank must run the same kernel plans: rank 0 decides and broadcasts (ops/autotune.py)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tune_worker, args=(r, world, port, str(tmp_path / "t.json"), q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for status, rank, payload in outs:
        assert status == "ok", payload
    res = {rank: payload for _, rank, payload in outs}
    for r in range(world):
        assert res[r][0] == (1, 10), res[r]  # rank 0's decision everywhere
        assert res[r][1] == r


def test_autotune_table_persists(tmp_path, monkeypatch):
    from jax_llama_amd.ops import autotune
    path = tmp_path / "tune.json"
    monkeypatch.setenv("JLA_TUNE_FILE", str(path))
    monkeypatch.setattr(autotune, "_PERSISTED", {})
    monkeypatch.setitem(autotune._LOADED, "done", False)
    key = (16, 6144, 4096, 3, torch.bfloat16, False, False)
    autotune._save("gemv", key, 9)
    autotune._save("gemm", (2048, 4096, 4096, 1, False), (2, 1))
    monkeypatch.setattr(autotune, "_PERSISTED", {})
    monkeypatch.setitem(autotune._LOADED, "done", False)
    assert autotune._persisted("gemv", key) == 9
    assert autotune._persisted("gemm", (2048, 4096, 4096, 1, False)) == (2, 1)
    assert autotune._persisted("gemm", (1, 2, 3, 0, False)) is None


def test_fused_row_parallel_routing():
    """Which row-parallel path a decode projection takes (parallel/comm.py linear_residual_, fused_o_state): the GEMV's
    fused epilogue up to 64 rows, the tiled GEMM's fused split-K reduce past them while the output fits the instance's
    exchange regions (one per 4096 elements; ranks sharing a device: all their workgroups resident at once), else
    nothing (the caller's partial + collective); the fused decode launch's o projection exchanges through the same
    instance (0 at world 1). Routing only: the kernels are GPU-tested (test_tp_gpu.py, test_kernels_gpu.py)."""
    from jax_llama_amd.parallel.comm import TPComm
    from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce

    calls = []

    class FakeFused(CustomAllReduce):
        def __init__(self, max_bytes, share=1):  # no device state: the capability checks are host arithmetic
            self.max_bytes, self.share, self.state, self.failed = max_bytes, share, 7, False

        def linear_residual_(self, *a, **k):
            calls.append("gemv")

        def tiled_residual_(self, *a, **k):
            calls.append("tiled")
            return True

    class W:
        n, k = 8192, 3584

    f = FakeFused(CustomAllReduce.fused_bytes(8192))
    assert f.can_fuse(64, 8192) and not f.can_fuse(65, 8192)
    assert f.can_fuse_tiled(256, 8192) and not f.can_fuse_tiled(257, 8192)  # 512 regions of 16 KiB = 8 MiB
    assert not FakeFused(CustomAllReduce.fused_bytes(8192), share=2).can_fuse_tiled(256, 8192)
    assert FakeFused(CustomAllReduce.fused_bytes(8192), share=2).can_fuse_tiled(64, 4096)
    comm = TPComm(size=8, rank=0, group=None, custom=None, reduce_dtype=torch.bfloat16, fused=f)

    class X:  # a decode activation's attributes as the routing reads them
        is_cuda, dtype = True, torch.bfloat16

        def __init__(self, m):
            self.shape = (m, 3584)

    for m, want in ((1, "gemv"), (64, "gemv"), (128, "tiled"), (256, "tiled")):
        calls.clear()
        assert comm.linear_residual_(X(m), W(), None, None) is True and calls == [want], (m, calls)
    calls.clear()
    assert comm.linear_residual_(X(300), W(), None, None) is False and calls == []
    assert comm.fused_o_state(X(1), W()) == 7
    assert TPComm(size=1, rank=0, group=None).fused_o_state(X(1), W()) == 0
    assert TPComm(size=8, rank=0, group=None, custom=None, reduce_dtype=torch.bfloat16,
                  fused=None).fused_o_state(X(1), W()) is None
