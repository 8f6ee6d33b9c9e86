"""One-shot push all-reduce over xGMI for decode-sized tensor-parallel messages.

SURVEY D1: RCCL (``torch.distributed`` backend ``nccl``) carries init, large messages and is the
correctness oracle; the 2 row-parallel all-reduces per layer per token (reference
``partition.py:67,70``: XLA inserts them after ``wo`` and ``w2``) are latency-bound, a few KiB to a
few MiB, so they go through ``csrc/kernels/allreduce.hip``: every rank pushes its input into every
peer's uncached, IPC-mapped receive slot over its direct xGMI link, raises a per-block flag, waits
for its peers' flags and sums the slots in rank order (bit-identical on every rank). One kernel,
no host sync, graph-capturable.

Rendezvous: each rank allocates its buffers, the IPC handles are exchanged with
``all_gather_object`` on the TP group, then every rank maps its peers'.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import ext


class CustomAllReduce:
    DTYPES = (torch.bfloat16, torch.float32)

    def __init__(self, state: int, rank: int, world: int, max_bytes: int):
        self.state = state
        self.rank = rank
        self.world = world
        self.max_bytes = max_bytes

    @classmethod
    def create(cls, ctx, max_bytes: int = 8 << 20, group=None) -> "CustomAllReduce":
        return cls.create_for(ctx.tp_rank, ctx.tp_size, ctx.tp_group if group is None else group, max_bytes)

    @classmethod
    def create_for(cls, rank: int, world: int, group, max_bytes: int = 8 << 20) -> "CustomAllReduce":
        if world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI hop)")
        max_bytes = (max_bytes + 15) // 16 * 16
        e = ext()
        buf, sig, hbuf, hsig = e.car_alloc(max_bytes, world)
        handles = [None] * world
        dist.all_gather_object(handles, (bytes(hbuf), bytes(hsig)), group=group)
        state = e.car_init(rank, world, max_bytes, buf, sig, [h[0] for h in handles], [h[1] for h in handles])
        dist.barrier(group=group)
        return cls(state, rank, world, max_bytes)

    def can_handle(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and t.dtype in self.DTYPES and 0 < nbytes <= self.max_bytes
                and nbytes % 16 == 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        ext().car_allreduce(self.state, t, t)
        return t

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty_like(t)
        ext().car_allreduce(self.state, t, out)
        return out

    def error(self) -> int:
        """1 if a kernel gave up waiting for a peer (bounded spin) since creation."""
        return int(ext().car_error(self.state))

    def close(self):
        if self.state:
            ext().car_destroy(self.state)
            self.state = 0
