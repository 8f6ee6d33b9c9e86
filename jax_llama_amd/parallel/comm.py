"""Tensor-parallel collectives.

The reference never calls a collective itself: XLA's GSPMD inserts the all-reduce after the
row-parallel ``wo``/``w2`` (``partition.py:67,70``) and the gathers for the vocab-parallel
``lm_head`` (``partition.py:77``). Here they are explicit:

  * ``all_reduce_residual_(partial, h, hb)``: the row-parallel sum of a projection's partial
    output, added to the fp32 residual stream ``h`` with its bf16 mirror ``hb`` rewritten — one
    kernel on the custom xGMI path (``csrc/kernels/allreduce.hip``), RCCL/gloo + an add otherwise;
  * ``argmax(val, idx, v_local)`` / ``gather_topk(vals, idx)``: the vocab-parallel sampler's
    gathers (greedy ``(max, argmax)`` pair per row; per-rank top-k candidates);
  * ``all_reduce_`` / ``all_gather``: generic sum / stack (prefill-sized messages, logits gathers).

On GPUs every decode-sized message goes through the custom one-/two-shot kernels (graph-capturable,
no host sync); larger messages and CPU/gloo runs use ``torch.distributed`` (RCCL / gloo).
``reduce_dtype`` is the dtype of the row-parallel partials on the wire: bf16 (default, half the bytes;
accumulated in fp32) or fp32 (``JLA_TP_REDUCE_DTYPE=fp32``).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


# GEMV-fused row-parallel all-reduce at decode (csrc/kernels/gemv.hip MODE_TPRESID); JLA_TP_FUSED=0: a separate
# collective kernel after each row-parallel GEMV
FUSED = os.environ.get("JLA_TP_FUSED", "1") != "0"
# ... and past the GEMV's 64 rows, in the tiled GEMM's split-K reduce (gemm.hip gemm_reduce_tp_kernel);
# JLA_TP_FUSED_TILED=0: GEMM partial + the collective kernel
FUSED_TILED = os.environ.get("JLA_TP_FUSED_TILED", "1") != "0"
# prefill-sized row-parallel partials over RCCL in bf16 (half the bytes, bf16 accumulation) instead of fp32
RCCL_BF16 = os.environ.get("JLA_TP_RCCL_BF16", "0") == "1"


def _default_reduce_dtype():
    return torch.float32 if os.environ.get("JLA_TP_REDUCE_DTYPE", "bf16") == "fp32" else torch.bfloat16


class TPComm:
    def __init__(self, size: int = 1, rank: int = 0, group=None, custom=None,
                 reduce_dtype: Optional[torch.dtype] = None, fused=None):
        self.size = size
        self.rank = rank
        self.group = group
        self.custom = custom  # parallel.custom_allreduce.CustomAllReduce or None
        self.reduce_dtype = reduce_dtype or _default_reduce_dtype()
        # a second custom instance reserved for the GEMV-fused row-parallel all-reduce (its per-workgroup counters
        # and slots must not interleave with the standalone collectives'); None: the standalone path only
        self.fused = fused

    @classmethod
    def from_context(cls, ctx, use_custom: bool = True, max_bytes: int = 16 << 20,
                     reduce_dtype: Optional[torch.dtype] = None, timeout_s: float = 10.0,
                     fused_hidden: Optional[int] = None) -> "TPComm":
        """``fused_hidden``: hidden size of the model, to size the GEMV-fused row-parallel all-reduce (``FUSED``;
        default 16384 columns)."""
        custom = fused = None
        if ctx.tp_size > 1 and ctx.device.type == "cuda" and use_custom:
            try:
                from .custom_allreduce import CustomAllReduce
            except ImportError:  # kernels not built: RCCL handles every message
                CustomAllReduce = None
            if CustomAllReduce is not None:
                from .custom_allreduce import CustomAllReduceError
                try:
                    custom = CustomAllReduce.create(ctx, max_bytes=max_bytes, timeout_s=timeout_s)
                except CustomAllReduceError as ex:  # same verdict on every rank: all fall back to RCCL
                    import logging
                    logging.getLogger(__name__).warning("custom all-reduce disabled: %s", ex)
                    custom = None
                if custom is not None and FUSED:
                    try:
                        fused = CustomAllReduce.create(ctx, max_bytes=CustomAllReduce.fused_bytes(
                            fused_hidden or 16384), timeout_s=timeout_s, kind="fused")
                    except CustomAllReduceError as ex:
                        import logging
                        logging.getLogger(__name__).warning("fused row-parallel all-reduce disabled: %s", ex)
                        fused = None
        if reduce_dtype is None and ctx.device.type != "cuda":
            reduce_dtype = torch.float32  # CPU (gloo) runs: the oracle-comparison path keeps fp32 partials
        return cls(ctx.tp_size, ctx.tp_rank, ctx.tp_group, custom, reduce_dtype, fused)

    def _host_staged(self, t: torch.Tensor) -> bool:
        # GPU tensors over a gloo group (multi-process tests sharing one GPU): stage through the host
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    # ------------------------------------------------------------------ sums
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

    def partial_dtype(self, numel: int, is_cuda: bool) -> torch.dtype:
        """The dtype a row-parallel GEMM should write its ``numel``-element partial in: ``reduce_dtype`` when the
        custom kernels take it (they sum bf16 partials in fp32 themselves), else fp32 whenever
        ``all_reduce_residual_`` would upcast a bf16 partial anyway -- the GEMM's fp32 store replaces the bf16
        rounding, the upcast copy and its allocation (the bytes on the wire are the same)."""
        dt = self.reduce_dtype
        if dt != torch.bfloat16 or self.size == 1:
            return dt
        c = self.custom
        if c is not None and is_cuda and 0 < numel * 2 <= c.max_bytes and (numel * 2) % 16 == 0:
            return dt
        return dt if (RCCL_BF16 and is_cuda and dist.get_backend(self.group) != "gloo") else torch.float32

    def all_reduce_residual_(self, partial: torch.Tensor, h: torch.Tensor, hb: Optional[torch.Tensor],
                             hb_pack: Optional[torch.Tensor] = None, owned: bool = False):
        """``h (fp32) += sum over ranks of partial``; ``hb = bf16(h)`` when given; ``hb_pack``: a packed-layout
        copy of hb too (custom path only -- callers ask ``packs_residual`` first). ``owned``: the caller's partial
        is scratch and may be reduced in place."""
        if self.size > 1 and self.custom is not None and hb is not None and self.custom.can_handle(partial):
            self.custom.all_reduce_residual_(partial, h, hb, hb_pack=hb_pack)
            return h
        if hb_pack is not None:
            raise RuntimeError("all_reduce_residual_: the packed hb copy needs the custom all-reduce path")
        # prefill-sized messages go over RCCL / gloo, which accumulate in the dtype on the wire: bf16 partials are
        # upcast so the sum is an fp32 sum like the custom kernels' (a bf16 ring sum would round up to world-1 times,
        # in an order RCCL picks); RCCL_BF16 (JLA_TP_RCCL_BF16=1) keeps them bf16 for half the bytes. Then ONE kernel
        # adds the sum into h and rewrites the mirror (ops.residual_add_)
        if self.size > 1:
            p = partial if partial.is_contiguous() else partial.contiguous()
            if p.dtype == torch.bfloat16 and not (RCCL_BF16 and p.is_cuda and not self._host_staged(p)):
                p = p.float()
            elif p.data_ptr() == partial.data_ptr() and not owned:
                p = p.clone()  # never reduce the caller's buffer in place
            self.all_reduce_(p)
        else:
            p = partial
        from .. import ops
        ops.residual_add_(h, p.view_as(h), hb)
        return h

    def linear_residual_(self, x: torch.Tensor, w, h: torch.Tensor, hb: torch.Tensor,
                         x_packed: Optional[torch.Tensor] = None, hb_pack: Optional[torch.Tensor] = None) -> bool:
        """The row-parallel projection + its all-reduce as ONE kernel when the fused path applies (decode rows,
        bf16 partials, a reserved instance): ``h += sum_ranks(x @ W^T)``, ``hb = bf16(h)``. Returns False (nothing
        done) otherwise -- the caller then runs ``linear`` + ``all_reduce_residual_``."""
        f = self.fused
        if (f is None or self.size == 1 or self.reduce_dtype != torch.bfloat16 or not x.is_cuda
                or x.dtype != torch.bfloat16):
            return False
        m = x.shape[0]
        if f.can_fuse(m, w.n):
            f.linear_residual_(x, w, h, hb, x_packed=x_packed, hb_pack=hb_pack)
            return True
        # past the GEMV's rows: the tiled GEMM's split-K reduce runs the exchange (when its plan splits K)
        if FUSED_TILED and hb_pack is None and m > 64 and f.can_fuse_tiled(m, w.n):
            return f.tiled_residual_(x, w, h, hb)
        return False

    def fused_o_state(self, x: torch.Tensor, w) -> Optional[int]:
        """The custom all-reduce state a fused decode launch's o projection exchanges its partials through (the GEMV
        epilogue's granule exchange, as ``linear_residual_``): 0 at world 1 (plain residual epilogue), None when the
        fused path does not apply (then the o projection runs through ``linear_residual_`` / the two-step path)."""
        if self.size == 1:
            return 0
        f = self.fused
        if (f is None or self.reduce_dtype != torch.bfloat16 or not x.is_cuda or x.dtype != torch.bfloat16
                or not f.can_fuse(x.shape[0], w.n)):
            return None
        return f._live()

    def packs_residual(self, nbytes: int) -> bool:
        """Whether ``all_reduce_residual_`` of an ``nbytes`` partial can also write a packed hb copy."""
        return self.size == 1 or (self.custom is not None and 0 < nbytes <= self.custom.max_bytes and nbytes % 16 == 0)

    # ------------------------------------------------------------------ sampler gathers
    def argmax(self, val: torch.Tensor, idx: torch.Tensor, v_local: int) -> torch.Tensor:
        """Global greedy token per row from every rank's local ``(max, argmax)`` (first max in rank
        order == smallest global index among ties, like ``jnp.argmax`` over the full vocab)."""
        if self.size == 1:
            return idx
        off = self.rank * v_local
        if self.custom is not None and val.is_cuda and self.custom.can_handle_pairs(val.numel()):
            return self.custom.argmax_pairs(val.float(), idx.to(torch.int32), off)
        vals = self.all_gather(val.float())  # [tp, B]
        idxs = self.all_gather(idx.to(torch.int32) + off)
        best = vals.argmax(0)
        return idxs.gather(0, best[None]).squeeze(0).to(torch.int32)

    def gather_topk(self, vals: torch.Tensor, idx: torch.Tensor):
        """``[B, k]`` candidates (global indices) of every rank -> ``[B, tp * k]`` in rank order."""
        b, k = vals.shape
        if self.custom is not None and vals.is_cuda and self.custom.can_handle_pairs(vals.numel()):
            return self.custom.topk_pairs(vals, idx, 0)
        gv = self.all_gather(vals).permute(1, 0, 2).reshape(b, self.size * k).contiguous()
        gi = self.all_gather(idx).permute(1, 0, 2).reshape(b, self.size * k).contiguous()
        return gv, gi

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

    # ------------------------------------------------------------------ failure detection
    def litmus(self):
        """Which collective paths passed the creation litmus on this group's links (None: no custom instance)."""
        return {"collective": getattr(self.custom, "litmus", None), "fused": getattr(self.fused, "litmus", None)}

    def check(self):
        """Raise if a custom collective timed out waiting for a peer (bounded spins ->
        error). Called by the decode loop at its periodic host poll."""
        if self.custom is not None:
            self.custom.check()
        if self.fused is not None:
            self.fused.check()

    def close(self):
        for c in (self.custom, self.fused):
            if c is not None:
                c.close()
        self.custom = self.fused = None


NO_COMM = TPComm()


class TPRankProxyComm(TPComm):
    """One rank of a ``size``-way tensor-parallel group, alone on one GPU (``bench.py`` ``tp_rank_proxy``).

    The model built on it holds exactly rank 0's shards (column / row / vocab slices at the real per-rank shapes)
    and issues exactly the launches a TP rank issues: every per-token collective runs the same custom kernel
    (``csrc/kernels/allreduce.hip``) on a world-1 instance -- same push / flag barrier / rank-order sum / fused
    residual + mirror epilogue -- so the step's launch structure and the kernels' local cost are the real ones.
    What it leaves out is the xGMI link: peer writes and peer flags land in local memory. Larger messages (prefill)
    are the identity sum (the RCCL call is skipped). Not a correctness path: the numbers are one shard's."""

    def __init__(self, size: int, custom=None, reduce_dtype: Optional[torch.dtype] = None, fused=None):
        super().__init__(size=size, rank=0, group=None, custom=custom, reduce_dtype=reduce_dtype, fused=fused)

    @classmethod
    def create(cls, size: int, max_bytes: int = 16 << 20, fused_hidden: Optional[int] = None) -> "TPRankProxyComm":
        from .custom_allreduce import CustomAllReduce
        fused = CustomAllReduce.local(max_bytes=CustomAllReduce.fused_bytes(fused_hidden or 16384)) if FUSED else None
        return cls(size, CustomAllReduce.local(max_bytes=max_bytes), fused=fused)

    def _host_staged(self, t: torch.Tensor) -> bool:
        return False

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.custom is not None and self.custom.can_handle(t):
            self.custom.all_reduce_(t)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0).expand((self.size,) + tuple(t.shape)).contiguous()

    def argmax(self, val: torch.Tensor, idx: torch.Tensor, v_local: int) -> torch.Tensor:
        if self.custom is not None and val.is_cuda and self.custom.can_handle_pairs(val.numel()):
            return self.custom.argmax_pairs(val.float(), idx.to(torch.int32), 0)
        return idx.to(torch.int32)

    def gather_topk(self, vals: torch.Tensor, idx: torch.Tensor):
        if self.custom is not None and vals.is_cuda and self.custom.can_handle_pairs(vals.numel()):
            return self.custom.topk_pairs(vals, idx, 0)
        return vals, idx

