"""Process-group bootstrap: one process per GPU (SPMD), launched by ``torchrun``.

Reference: the library is single-process/multi-device (``jax_example.py:12-13`` builds a
``(1, n_devices)`` mesh, TP degree = every visible device); only its test harness is
multi-process (``jax_test.py:60-70``: ``init_process_group("nccl")``, ``set_device``).

Here every rank owns one GPU. ``WORLD_SIZE`` ranks are arranged as a ``(dp, tp)`` mesh:
ranks ``[d*tp, (d+1)*tp)`` form tensor-parallel group ``d`` (contiguous ranks = GPUs with
direct xGMI links on one node). Backend ``nccl`` is RCCL on ROCm; ``gloo`` for CPU runs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist


def env_rank_info():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local_rank


def init_distributed(backend: Optional[str] = None, device_type: Optional[str] = None,
                     timeout_s: int = 600) -> "ParallelContext":
    """Initialise torch.distributed from the torchrun environment (no-op for 1 process)."""
    rank, world, local_rank = env_rank_info()
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # JLA_SINGLE_DEVICE=1 (test hook): every rank shares GPU 0, e.g. to rehearse a multi-rank
        # launch on a one-GPU box (together with JLA_DIST_BACKEND=gloo: RCCL needs distinct GPUs)
        dev_idx = 0 if os.environ.get("JLA_SINGLE_DEVICE", "0") == "1" else local_rank
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = os.environ.get("JLA_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return ParallelContext(world=world, rank=rank, local_rank=local_rank, device=device)


@dataclass
class ParallelContext:
    world: int = 1
    rank: int = 0
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None

    def setup_mesh(self, tp: Optional[int] = None) -> "ParallelContext":
        """Split the world into ``world // tp`` data-parallel replicas of ``tp`` ranks."""
        tp = self.world if tp is None else tp
        if self.world % tp:
            raise ValueError(f"world size {self.world} not divisible by tp={tp}")
        self.tp_size, self.dp_size = tp, self.world // tp
        self.tp_rank, self.dp_rank = self.rank % tp, self.rank // tp
        if self.world > 1 and dist.is_initialized():
            for d in range(self.dp_size):  # every rank must create every group
                ranks = list(range(d * tp, (d + 1) * tp))
                g = dist.new_group(ranks) if tp > 1 else None
                if d == self.dp_rank:
                    self.tp_group = g
            if self.dp_size > 1:
                for t in range(tp):
                    ranks = list(range(t, self.world, tp))
                    g = dist.new_group(ranks)
                    if t == self.tp_rank:
                        self.dp_group = g
        return self

    def barrier(self):
        if self.world > 1 and dist.is_initialized():
            if self.device.type == "cuda" and dist.get_backend() == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_max(self, values):
        """Element-wise max over all ranks of a list of floats (host result)."""
        t = torch.tensor(values, dtype=torch.float64)
        if self.world > 1 and dist.is_initialized():
            if dist.get_backend() == "nccl":
                t = t.to(self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.cpu()]


def single_process_context(device="cpu") -> ParallelContext:
    d = torch.device(device)
    return ParallelContext(device=d, local_rank=d.index or 0)
