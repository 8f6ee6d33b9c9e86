"""Native checkpoint: save / reload a model in its DEPLOYED form (safetensors, per TP rank).

The reference only loads Meta ``.pth`` shards (``convert_weights.py:52-92``) and never saves
("Checkpoint / resume"). Converting a Meta checkpoint costs a host pass over
every tensor (slice per rank, transpose, fold the RMSNorm gains into the following projection),
which for 65B/70B takes minutes. ``save_pretrained`` writes what the kernels actually consume, so
``from_pretrained`` is one mmap + host-to-device copy per tensor:

    <dir>/config.json                      LLaMAConfig (HF-style)
    <dir>/jla_native.json                  {"format": 1, "tp": N, "norm_folded": true}
    <dir>/model-rank{r:02d}-of-{N:02d}.safetensors

Tensors per rank (bf16 unless noted; ``[n, k]`` = Meta ``[out, in]`` orientation, this rank's
shard, RMSNorm gains already folded into ``qkv``/``gate_up``/``lm_head`` columns):

    wte [V, D]                   ln_f [D] fp32
    h.{i}.qkv [(H+2Hkv)/tp*Dh, D]  h.{i}.o [D, H/tp*Dh]
    h.{i}.gate_up [2F/tp, D] (w1/w3 interleaved in 16-row tiles)   h.{i}.down [D, F/tp]
    h.{i}.attention_norm [D] fp32   h.{i}.ffn_norm [D] fp32        lm_head [V/tp, D]

Dense ``[n, k]`` is stored (not the MFMA fragment packing), so files are device-independent and the
reload into the packed GPU layout is exact (bit-for-bit the same weights). Reloading needs the
same TP degree; changing it goes through the Meta format (``utils.checkpoint``).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

from ..config import LLaMAConfig

FORMAT = 1


def _rank_file(directory: str, rank: int, size: int) -> str:
    return os.path.join(directory, f"model-rank{rank:02d}-of-{size:02d}.safetensors")


def save_pretrained(model, directory: str) -> str:
    """Write this rank's deployed weights (every TP rank calls it; rank 0 writes the metadata)."""
    from safetensors.torch import save_file

    os.makedirs(directory, exist_ok=True)
    rank, size = model.tp_rank, model.tp_size
    t = {"wte": model.wte, "ln_f": model.ln_f.float(), "lm_head": model.lm_head.dense()}
    for i, lw in enumerate(model.layers):
        t[f"h.{i}.qkv"] = lw.qkv.dense()
        t[f"h.{i}.o"] = lw.o.dense()
        t[f"h.{i}.gate_up"] = lw.gu.dense()
        t[f"h.{i}.down"] = lw.down.dense()
        t[f"h.{i}.attention_norm"] = lw.attention_norm.float()
        t[f"h.{i}.ffn_norm"] = lw.ffn_norm.float()
    t = {k: v.detach().to("cpu").contiguous() for k, v in t.items()}
    path = _rank_file(directory, rank, size)
    save_file(t, path, metadata={"format": str(FORMAT), "tp_rank": str(rank), "tp_size": str(size)})
    if rank == 0:
        model.config.save_pretrained(directory)
        with open(os.path.join(directory, "jla_native.json"), "w") as f:
            json.dump({"format": FORMAT, "tp": size, "norm_folded": True,
                       "num_hidden_layers": model.config.num_hidden_layers}, f)
    return path


def from_pretrained(directory: str, device="cpu", comm=None, config: Optional[LLaMAConfig] = None):
    """Rebuild a ``LLaMAForCausalLM`` from ``save_pretrained`` output for this TP rank."""
    from safetensors import safe_open

    from ..models.llama import LLaMAForCausalLM
    from ..models.weights import PackedLinear

    with open(os.path.join(directory, "jla_native.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"unsupported native checkpoint format {meta.get('format')}")
    cfg = config or LLaMAConfig.from_pretrained(directory)
    model = LLaMAForCausalLM(cfg, device=device, comm=comm, _do_init=False)
    if meta["tp"] != model.tp_size:
        raise ValueError(f"checkpoint was saved at tp={meta['tp']} but this model runs tp={model.tp_size}; "
                         "re-shard through the Meta format (utils.checkpoint.save_meta_checkpoint)")
    dev = model.device
    with safe_open(_rank_file(directory, model.tp_rank, model.tp_size), framework="pt", device="cpu") as f:
        def get(name, dtype=None):
            x = f.get_tensor(name)
            return x.to(dev, dtype) if dtype is not None else x.to(dev)

        model.wte = get("wte", torch.bfloat16).contiguous()
        model.ln_f = get("ln_f", torch.float32)
        model.lm_head = PackedLinear.from_dense(f.get_tensor("lm_head"), dev)
        for i, lw in enumerate(model.layers):
            lw.qkv = PackedLinear.from_dense(f.get_tensor(f"h.{i}.qkv"), dev)
            lw.o = PackedLinear.from_dense(f.get_tensor(f"h.{i}.o"), dev)
            lw.gu = PackedLinear.from_dense(f.get_tensor(f"h.{i}.gate_up"), dev)
            lw.down = PackedLinear.from_dense(f.get_tensor(f"h.{i}.down"), dev)
            lw.attention_norm = get(f"h.{i}.attention_norm", torch.float32)
            lw.ffn_norm = get(f"h.{i}.ffn_norm", torch.float32)
    return model
