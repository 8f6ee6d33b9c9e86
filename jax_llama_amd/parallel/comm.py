"""Tensor-parallel collectives.

The reference never calls a collective itself: XLA's GSPMD inserts the all-reduce after the
row-parallel ``wo``/``w2`` (``partition.py:67,70``) and the gathers for the vocab-parallel
``lm_head`` (``partition.py:77``). Here they are explicit:

  * ``all_reduce_``: sum over the TP group. On GPUs small (decode-sized) messages go through
    the custom one-shot xGMI all-reduce (``csrc/comm/allreduce.hip``: peer-mapped IPC
    buffers, every rank reads all peers over its direct links, graph-capturable); larger
    messages and CPU/gloo runs use ``torch.distributed`` (RCCL / gloo).
  * ``all_gather``: stacks every rank's tensor (sampler candidates, vocab-parallel logits).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


class TPComm:
    def __init__(self, size: int = 1, rank: int = 0, group=None, custom=None):
        self.size = size
        self.rank = rank
        self.group = group
        self.custom = custom  # parallel.custom_allreduce.CustomAllReduce or None

    @classmethod
    def from_context(cls, ctx, use_custom: bool = True, max_bytes: int = 8 << 20) -> "TPComm":
        custom = None
        if ctx.tp_size > 1 and ctx.device.type == "cuda" and use_custom:
            try:
                from .custom_allreduce import CustomAllReduce
            except ImportError:  # one-shot xGMI kernel not built: RCCL handles every message
                CustomAllReduce = None
            if CustomAllReduce is not None:
                custom = CustomAllReduce.create(ctx, max_bytes=max_bytes)
        return cls(ctx.tp_size, ctx.tp_rank, ctx.tp_group, custom)

    def _host_staged(self, t: torch.Tensor) -> bool:
        # GPU tensors over a gloo group (multi-process tests sharing one GPU): stage through the host
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return t
        if self.custom is not None and self.custom.can_handle(t):
            self.custom.all_reduce_(t)
            return t
        if self._host_staged(t):
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Returns ``[size, *t.shape]``."""
        if self.size == 1:
            return t.unsqueeze(0)
        src = t.contiguous().reshape(-1)
        staged = self._host_staged(t)
        if staged:
            src = src.cpu()
        # flat [size * numel] buffer: the layout both RCCL and gloo accept for all_gather_into_tensor
        out = torch.empty(self.size * t.numel(), dtype=t.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src, group=self.group)
        if staged:
            out = out.to(t.device)
        return out.view((self.size,) + tuple(t.shape))


NO_COMM = TPComm()
