"""Custom one-shot all-reduce (csrc/kernels/allreduce.hip) against the exact sum.

Two processes share the one GPU of the test box (IPC mapping between processes works the same on
one device as across xGMI peers; the cross-GPU link itself is exercised only on a multi-GPU node).
The handle exchange uses a gloo group (RCCL refuses two ranks on one device)."""
from __future__ import annotations

import multiprocessing as mp
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(rank, n, dtype, seed):
    g = torch.Generator().manual_seed(seed * 100 + rank)
    return (torch.randn(n, generator=g) * (rank + 1)).to(dtype)


CASES = [(8, torch.float32), (4096, torch.bfloat16), (16 * 4096, torch.bfloat16), (300_000, torch.float32),
         (512 * 4096, torch.bfloat16)]


def _check(y, n, dt, seed, world):
    want = sum(_inputs(r, n, dt, seed).float() for r in range(world))
    if dt == torch.bfloat16:
        torch.testing.assert_close(y.float(), want.to(dt).float(), rtol=1e-2, atol=1e-2)
    else:
        torch.testing.assert_close(y, want, rtol=1e-6, atol=1e-5)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
        car = CustomAllReduce.create_for(rank, world, None, max_bytes=8 << 20)
        digest = []
        for rep in range(3):  # repeated calls exercise both parity buffers and the epochs
            for i, (n, dt) in enumerate(CASES):
                x = _inputs(rank, n, dt, i + 10 * rep).cuda()
                assert car.can_handle(x)
                y = car.all_reduce(x).cpu()
                _check(y, n, dt, i + 10 * rep, world)
                digest.append(float(y.double().sum()))
        # graph capture + replay
        x = _inputs(rank, 4096 * 4, torch.bfloat16, 99).cuda()
        car.all_reduce_(x.clone())  # warm
        buf = x.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            car.all_reduce_(buf)
        buf.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        _check(buf.cpu(), 4096 * 4, torch.bfloat16, 99, world)
        assert car.error() == 0
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put(("ok", rank, digest))
    except Exception:  # pragma: no cover - surfaced in the parent
        import traceback
        q.put(("err", rank, traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_matches_sum(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = []
    try:
        for _ in range(world):
            outs.append(q.get(timeout=240))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for status, rank, payload in outs:
        assert status == "ok", payload
    # bit-identical on every rank (fixed summation order)
    digests = {rank: payload for _, rank, payload in outs}
    for r in range(1, world):
        assert digests[r] == digests[0]
