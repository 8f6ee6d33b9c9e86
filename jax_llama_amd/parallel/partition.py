"""Partition rules for tensor parallelism (reference ``jax_llama/partition.py``).

The reference feeds regex rules to GSPMD (``pjit``), which then inserts collectives. Here
the same rules drive *explicit* SPMD: ``shard_tree`` slices every parameter for one rank
(one process per GPU), and the model performs the two all-reduces per layer itself
(``parallel/comm.py``: RCCL or the custom xGMI all-reduce).

API parity:
  * ``get_partition_spec(tree, rules)`` — first matching rule wins, every leaf must match
    (``partition.py:10-41``).
  * ``get_llama_param_partition_spec(params, fsdp=False)`` (``partition.py:43-81``).
  * ``with_sharding_constraint`` / ``with_named_sharding_constraint`` (``partition.py:83-98``)
    are batch-split helpers: no-ops unless a data-parallel mesh with dp > 1 is given.
"""
from __future__ import annotations

import re
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import torch


class PartitionSpec(tuple):
    """Per-dimension mesh-axis names (``None`` = replicated), like ``jax.sharding.P``."""

    def __new__(cls, *axes):
        return super().__new__(cls, axes)

    def __repr__(self):
        return "P(" + ", ".join(repr(a) for a in self) + ")"


P = PartitionSpec
_UNMATCHED = object()


def flatten_tree(tree: Dict[str, Any], prefix: Tuple[str, ...] = ()) -> Dict[Tuple[str, ...], Any]:
    out = {}
    for k, v in tree.items():
        key = prefix + (str(k),)
        if isinstance(v, dict):
            out.update(flatten_tree(v, key))
        else:
            out[key] = v
    return out


def unflatten_tree(flat: Dict[Tuple[str, ...], Any]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for key, v in flat.items():
        d = out
        for k in key[:-1]:
            d = d.setdefault(k, {})
        d[key[-1]] = v
    return out


def _match(qs: Sequence[str], ks: Tuple[str, ...]) -> bool:
    """True if the regexes ``qs`` fully match some window of the key path ``ks``."""
    qts = [re.compile(q + "$") for q in qs]
    for i in range(len(ks) - len(qs) + 1):
        if all(q.match(k) for q, k in zip(qts, ks[i:])):
            return True
    return False


def get_partition_spec(in_dict: Dict[str, Any], rules: List[Tuple[Tuple[str, ...], PartitionSpec]]):
    flat = flatten_tree(in_dict)
    result = {}
    for key in flat:
        spec = _UNMATCHED
        for rule, replacement in rules:
            if _match(rule, key):
                spec = replacement
                break
        result[key] = spec
    if any(v is _UNMATCHED for v in result.values()):
        missing = [k for k, v in result.items() if v is _UNMATCHED]
        raise AssertionError(f"Incomplete partition spec: {missing[:4]}")
    return unflatten_tree(result)


def _get_partition_rules_llama(fsdp: bool = False):
    if fsdp:
        return [
            (("transformer", "wte", "embedding"), P("mp", "dp")),
            (("attention", "(wq|wk|wv)", "kernel"), P("dp", "mp")),
            (("attention", "wo", "kernel"), P("mp", "dp")),
            (("feed_forward", "w1", "kernel"), P("dp", "mp")),
            (("feed_forward", "w2", "kernel"), P("mp", "dp")),
            (("feed_forward", "w3", "kernel"), P("dp", "mp")),
            (("attention_norm", "kernel"), P(None)),
            (("ffn_norm", "kernel"), P(None)),
            (("transformer", "ln_f", "kernel"), P(None)),
            (("lm_head", "kernel"), P("dp", "mp")),
        ]
    return [
        (("transformer", "wte", "embedding"), P("mp", None)),
        (("attention", "(wq|wk|wv)", "kernel"), P(None, "mp")),
        (("attention", "wo", "kernel"), P("mp", None)),
        (("feed_forward", "w1", "kernel"), P(None, "mp")),
        (("feed_forward", "w2", "kernel"), P("mp", None)),
        (("feed_forward", "w3", "kernel"), P(None, "mp")),
        (("attention_norm", "kernel"), P(None)),
        (("ffn_norm", "kernel"), P(None)),
        (("transformer", "ln_f", "kernel"), P(None)),
        (("lm_head", "kernel"), P(None, "mp")),
    ]


def get_llama_param_partition_spec(params: Dict[str, Any], fsdp: bool = False):
    return get_partition_spec(params, _get_partition_rules_llama(fsdp=fsdp))


def shard_tensor(x, spec: PartitionSpec, rank: int, size: int, axis_name: str = "mp"):
    """Slice ``x`` for ``rank`` along every dim whose spec names ``axis_name``."""
    if size == 1:
        return x
    for dim, ax in enumerate(spec):
        if ax == axis_name:
            n = x.shape[dim]
            if n % size:
                raise ValueError(f"dim {dim} of size {n} not divisible by tp={size}")
            c = n // size
            x = x.narrow(dim, rank * c, c)
    return x


def shard_tree(params: Dict[str, Any], rank: int, size: int, fsdp: bool = False,
               replicate_embedding: bool = True):
    """Return this rank's shard of every parameter (views where possible).

    ``replicate_embedding``: the reference vocab-shards ``wte`` (``partition.py:64``); we
    keep the (small) table replicated so the lookup needs no collective.
    """
    specs = flatten_tree(get_llama_param_partition_spec(params, fsdp=fsdp))
    flat = flatten_tree(params)
    out = {}
    for key, x in flat.items():
        spec = specs[key]
        if replicate_embedding and key[-2:] == ("wte", "embedding"):
            spec = P(None, None)
        out[key] = shard_tensor(x, spec, rank, size)
    return unflatten_tree(out)


# ----------------------------------------------------------------------------------
# Batch (dp) sharding constraints — reference partition.py:83-98 / generation.py:25-26,44
# ----------------------------------------------------------------------------------
class Mesh:
    """A (dp, mp) process mesh: ``dp`` replicas, each a TP group of ``mp`` ranks."""

    def __init__(self, dp: int = 1, mp: int = 1, rank: int = 0, dp_group=None):
        self.shape = {"dp": dp, "mp": mp}
        self.dp_rank = rank // mp
        self.mp_rank = rank % mp
        self.dp_group = dp_group  # torch.distributed group of this rank's dp peers (same mp rank)

    @classmethod
    def from_context(cls, ctx) -> "Mesh":
        return cls(dp=ctx.dp_size, mp=ctx.tp_size, rank=ctx.rank, dp_group=ctx.dp_group)

    @property
    def devices(self):
        return self.shape


def gather_dp(x, mesh: Optional[Mesh]):
    """Inverse of the dp batch split: all-gather every dp replica's rows (dim 0) when a process
    group is available; otherwise return this replica's rows unchanged."""
    if mesh is None or mesh.shape["dp"] == 1 or not torch.is_tensor(x):
        return x
    import torch.distributed as dist
    if not dist.is_initialized():
        return x
    dp = mesh.shape["dp"]
    xs = x.contiguous()
    staged = xs.is_cuda and dist.get_backend(mesh.dp_group) == "gloo"
    src = xs.cpu() if staged else xs
    out = [torch.empty_like(src) for _ in range(dp)]
    dist.all_gather(out, src, group=mesh.dp_group)
    full = torch.cat(out, 0)
    return full.to(x.device) if staged else full


def with_sharding_constraint(x, axis_resources):
    """No-op outside a mesh context (as the reference on CPU / without pjit)."""
    return x


def with_named_sharding_constraint(x, mesh: Optional[Mesh], partition_spec: PartitionSpec):
    """Keep this dp-rank's slice of the batch dim when ``mesh`` has dp > 1."""
    if mesh is None or mesh.shape["dp"] == 1 or not torch.is_tensor(x):
        return x
    if len(partition_spec) and partition_spec[0] == "dp":
        dp = mesh.shape["dp"]
        n = x.shape[0]
        if n % dp == 0:
            c = n // dp
            return x.narrow(0, mesh.dp_rank * c, c)
    return x
