"""Weight containers.

On the GPU every linear weight lives in the *MFMA fragment-packed* layout
(``ops.reference.pack_frag16x32``): a ``[N, K]`` matrix becomes
``[N/16][K/32][64 lanes][8 bf16]`` so that each 16(n) x 32(k) block — exactly the B
operand of one ``v_mfma_f32_16x16x32_bf16`` — is one contiguous 1 KiB run that a wave loads
with a single ``global_load_dwordx4`` (16 B/lane, perfectly coalesced) and that an LDS-DMA
copy lands lane-linearly (bank-conflict-free ``ds_read_b128``). Both the decode GEMV-like
kernel and the prefill GEMM consume this one layout, so weights are stored once.

Norm weights are folded into the following projection at load time
(``W'[n, k] = W[n, k] * g[k]``), so RMSNorm reduces to a per-row ``inv_rms`` scale that the
GEMM applies in its epilogue (reference RMSNorm: ``model.py:28-48``).

On the CPU (test/oracle path) the same object simply holds the dense ``[N, K]`` bf16 matrix.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import reference as ref

BF16 = torch.bfloat16


class PackedLinear:
    """``y = x @ W^T`` with ``W`` logically ``[n, k]`` (Meta ``[out, in]`` orientation)."""

    def __init__(self, weight: torch.Tensor, n: int, k: int):
        self.weight = weight
        self.n = n
        self.k = k

    @property
    def device(self) -> torch.device:
        return self.weight.device

    @property
    def packed(self) -> bool:
        return self.weight.dim() == 4

    @classmethod
    def from_dense(cls, w: torch.Tensor, device, fold: Optional[torch.Tensor] = None) -> "PackedLinear":
        n, k = w.shape
        device = torch.device(device)
        src = w.to(device)
        if fold is not None:
            src = (src.float() * fold.to(device).float()[None, :])
        src = src.to(BF16)
        if device.type == "cuda":
            if n % 16 or k % 32:
                raise ValueError(f"GPU linear weights need N%16==0 and K%32==0, got {n}x{k}")
            return cls(ref.pack_frag16x32(src), n, k)
        return cls(src.contiguous(), n, k)

    @classmethod
    def random(cls, n: int, k: int, device, std: float = 0.02, generator=None) -> "PackedLinear":
        """Random-init directly in the on-device layout (synthetic benchmarks)."""
        device = torch.device(device)
        if device.type == "cuda":
            w = torch.empty(n // 16, k // 32, 64, 8, dtype=BF16, device=device)
        else:
            w = torch.empty(n, k, dtype=BF16, device=device)
        w.normal_(0.0, std, generator=generator)
        return cls(w, n, k)

    def dense(self) -> torch.Tensor:
        """The ``[n, k]`` bf16 matrix (unpacks on the GPU; used for debugging / oracles)."""
        if self.packed:
            return ref.unpack_frag16x32(self.weight, self.n, self.k)
        return self.weight

    def nbytes(self) -> int:
        return self.weight.numel() * self.weight.element_size()
