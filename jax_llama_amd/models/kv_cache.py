"""Static, pre-allocated KV cache.

Reference: Flax ``"cache"`` collection created by ``init_cache`` (``model.py:459-476``) and
updated by ``_concatenate_to_cache`` (``model.py:169-199``): per layer ``cached_key`` /
``cached_value`` of shape ``(B, T_max, Hkv, Dh)`` holding post-RoPE keys, plus a scalar
``cache_index`` advanced by the number of tokens written.

Here: two tensors ``[L, B, Hkv_local, T_max, Dh]`` (bf16) so that one (b, kv-head)'s keys
are a single contiguous ``T x 256 B`` run — the decode attention kernel streams it with
1 KiB-per-wave-instruction loads — and the slot index is mirrored in a device int32 so
hipGraph-captured decode steps read/advance it without host round trips. No forward pass
is run to create it (unlike the reference's ``module.init`` trick).
"""
from __future__ import annotations

import torch


class KVCache:
    def __init__(self, num_layers: int, batch_size: int, num_kv_heads: int, max_length: int,
                 head_dim: int, device, dtype=torch.bfloat16):
        device = torch.device(device)
        shape = (num_layers, batch_size, num_kv_heads, max_length, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        self.batch_size = batch_size
        self.max_length = max_length
        self.index = 0  # host mirror of the number of filled slots
        self.index_t = torch.zeros(1, dtype=torch.int32, device=device)

    @property
    def device(self):
        return self.k.device

    def layer(self, i: int):
        return self.k[i], self.v[i]

    def advance(self, n: int) -> None:
        self.index += n
        self.index_t.add_(n)

    def reset(self) -> None:
        self.index = 0
        self.index_t.zero_()

    def rows(self, b0: int, b1: int) -> "KVCacheRows":
        """The cache of batch rows ``[b0, b1)`` (every layer): a view whose per-layer K / V are contiguous slices, for a
        prefill run in row chunks (runtime/engine.py)."""
        return KVCacheRows(self, b0, b1)

    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()

    # Flax-cache-like view for API parity / debugging (per-layer dict, (B, T, Hkv, Dh)).
    def as_dict(self):
        return {
            str(i): {
                "cached_key": self.k[i].permute(0, 2, 1, 3),
                "cached_value": self.v[i].permute(0, 2, 1, 3),
                "cache_index": self.index,
            }
            for i in range(self.k.shape[0])
        }


class KVCacheRows:
    """Rows ``[b0, b1)`` of a KVCache: ``layer(i)`` gives contiguous ``[b1 - b0, Hkv, T, Dh]`` views; the slot index is
    the parent's (one position for every row)."""

    def __init__(self, parent: KVCache, b0: int, b1: int):
        self.parent = parent
        self.b0, self.b1 = b0, b1
        self.batch_size = b1 - b0
        self.max_length = parent.max_length

    @property
    def device(self):
        return self.parent.device

    @property
    def index(self):
        return self.parent.index

    @property
    def index_t(self):
        return self.parent.index_t

    def layer(self, i: int):
        return self.parent.k[i, self.b0:self.b1], self.parent.v[i, self.b0:self.b1]
