"""Meta checkpoint I/O.

``convert_llama_weights`` keeps the reference signature and output
(``/root/reference/jax_llama/convert_weights.py:52-92``): it reads ``consolidated.XX.pth``
shards (sorted by the XX index) plus ``params.json``, merges Meta's model-parallel shards
along the same axes as the reference and returns ``(params, LLaMAConfig)`` where ``params``
is the reference-named tree with Flax ``(in, out)`` kernel orientation:

    transformer.wte.embedding (V, D)          transformer.ln_f.kernel (D,)
    transformer.h.{i}.attention.{wq,wk,wv,wo}.kernel
    transformer.h.{i}.feed_forward.{w1,w2,w3}.kernel
    transformer.h.{i}.{attention_norm,ffn_norm}.kernel
    lm_head.kernel (D, V)

Differences (MI355X-first, documented):
  * shards are opened with ``torch.load(mmap=True, weights_only=True)`` — nothing is
    unpickled beyond tensors and nothing is materialised until a rank slices it; a
    single-shard checkpoint yields zero-copy transposed *views*;
  * tensors keep the checkpoint dtype (bf16) instead of being widened to fp32 (the
    reference's fp32 copies need several hundred GB of host RAM for 65B/70B); pass
    ``dtype=torch.float32`` for the reference behaviour;
  * the embedding merge axis is inferred from the shard shapes (LLaMA-1/2
    ``ParallelEmbedding`` splits the model dim, Llama-3 ``VocabParallelEmbedding`` splits the
    vocab; the reference's fixed ``axis=1`` is only right for the former);
  * ``params.json`` keys unknown to ``ModelArgs`` are tolerated (``use_scaled_rope`` of
    Llama-3.1 enables the scaled RoPE table) unless ``strict=True``.
"""
from __future__ import annotations

import json
import logging
import os
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import torch

from ..config import LLaMAConfig, ModelArgs, config_from_params

logger = logging.getLogger(__name__)

# Meta TP split axis of each per-layer tensor ([out, in] orientation).
_COL = ("attention.wq", "attention.wk", "attention.wv", "feed_forward.w1", "feed_forward.w3")
_ROW = ("attention.wo", "feed_forward.w2")


def _load_shard(path: Path):
    try:
        return torch.load(path, map_location="cpu", mmap=True, weights_only=True)
    except RuntimeError:
        # legacy (non-zipfile) serialisation cannot be mmapped
        return torch.load(path, map_location="cpu", weights_only=True)


def load_meta_shards(ckpt_dir: Union[str, Path], verbose: bool = False) -> Tuple[List[Dict], Dict]:
    ckpt_dir = Path(ckpt_dir)
    paths = sorted(ckpt_dir.glob("*.pth"))
    if not paths:
        raise FileNotFoundError(f"no *.pth shards in {ckpt_dir}")
    shards = {}
    for i, p in enumerate(paths):
        if verbose:
            print(f"Loading checkpoint {i + 1} of {len(paths)} ...")
        shards[int(p.name.split(".", maxsplit=2)[1])] = _load_shard(p)
    ordered = [shards[i] for i in sorted(shards)]
    with open(ckpt_dir / "params.json") as f:
        params = json.load(f)
    return ordered, params


def _cat(ts: List[torch.Tensor], axis: int, dtype) -> torch.Tensor:
    t = ts[0] if len(ts) == 1 else torch.cat(ts, axis)
    return t if dtype is None else t.to(dtype)


def merge_meta_shards(shards: List[Dict], n_layers: int, dtype=None) -> Dict[str, torch.Tensor]:
    """Merge Meta MP shards into one Meta-layout state dict ([out, in] weights)."""
    n = len(shards)
    out: Dict[str, torch.Tensor] = {}
    emb = [s["tok_embeddings.weight"] for s in shards]
    if n > 1:
        d_s, v_s = emb[0].shape[1], emb[0].shape[0]
        # LLaMA-1/2 ParallelEmbedding: split on dim (axis 1); Llama-3: split on vocab (axis 0)
        axis = 1 if all(e.shape[0] == v_s for e in emb) and shards[0]["norm.weight"].shape[0] == d_s * n else 0
    else:
        axis = 0
    out["tok_embeddings.weight"] = _cat(emb, axis, dtype)
    out["norm.weight"] = _cat([shards[0]["norm.weight"]], 0, dtype)
    out["output.weight"] = _cat([s["output.weight"] for s in shards], 0, dtype)
    for i in range(n_layers):
        pre = f"layers.{i}."
        for name in _COL:
            out[pre + name + ".weight"] = _cat([s[pre + name + ".weight"] for s in shards], 0, dtype)
        for name in _ROW:
            out[pre + name + ".weight"] = _cat([s[pre + name + ".weight"] for s in shards], 1, dtype)
        for name in ("attention_norm", "ffn_norm"):
            out[pre + name + ".weight"] = _cat([shards[0][pre + name + ".weight"]], 0, dtype)
    return out


def meta_state_dict_to_params(sd: Dict[str, torch.Tensor], n_layers: int) -> Dict:
    """Meta-layout state dict -> reference-named tree (``(in, out)`` transposed views)."""
    h = {}
    for i in range(n_layers):
        pre = f"layers.{i}."
        h[str(i)] = {
            "attention": {k: {"kernel": sd[pre + f"attention.{k}.weight"].t()} for k in ("wq", "wk", "wv", "wo")},
            "feed_forward": {k: {"kernel": sd[pre + f"feed_forward.{k}.weight"].t()} for k in ("w1", "w2", "w3")},
            "attention_norm": {"kernel": sd[pre + "attention_norm.weight"]},
            "ffn_norm": {"kernel": sd[pre + "ffn_norm.weight"]},
        }
    return {
        "transformer": {
            "wte": {"embedding": sd["tok_embeddings.weight"]},
            "ln_f": {"kernel": sd["norm.weight"]},
            "h": h,
        },
        "lm_head": {"kernel": sd["output.weight"].t()},
    }


def params_to_meta_state_dict(params: Dict) -> Dict[str, torch.Tensor]:
    tr = params["transformer"]
    sd = {"tok_embeddings.weight": torch.as_tensor(tr["wte"]["embedding"]),
          "norm.weight": torch.as_tensor(tr["ln_f"]["kernel"]),
          "output.weight": torch.as_tensor(params["lm_head"]["kernel"]).t()}
    for i, blk in tr["h"].items():
        pre = f"layers.{i}."
        for k in ("wq", "wk", "wv", "wo"):
            sd[pre + f"attention.{k}.weight"] = torch.as_tensor(blk["attention"][k]["kernel"]).t()
        for k in ("w1", "w2", "w3"):
            sd[pre + f"feed_forward.{k}.weight"] = torch.as_tensor(blk["feed_forward"][k]["kernel"]).t()
        sd[pre + "attention_norm.weight"] = torch.as_tensor(blk["attention_norm"]["kernel"])
        sd[pre + "ffn_norm.weight"] = torch.as_tensor(blk["ffn_norm"]["kernel"])
    return sd


def config_from_params_json(params: Dict, vocab_size: int, max_seq_len: int, strict: bool = False) -> LLaMAConfig:
    p = dict(params)
    p.update({"vocab_size": vocab_size, "max_seq_len": max_seq_len})
    extra = {}
    if not strict:
        known = set(ModelArgs.__dataclass_fields__)
        extra = {k: p.pop(k) for k in list(p) if k not in known}
        if extra:
            logger.info("params.json keys not in ModelArgs: %s", sorted(extra))
    cfg = config_from_params(ModelArgs(**p))
    if extra.get("use_scaled_rope"):
        cfg.use_scaled_rope = True
    return cfg


def convert_llama_weights(ckpt_dir: str, tokenizer, max_seq_len: int = 2048, verbose: bool = False,
                          dtype: Optional[torch.dtype] = None, strict: bool = False):
    """Reference ``convert_llama_weights`` (``convert_weights.py:52``). ``tokenizer`` may be
    a tokenizer (``len()`` gives the vocab) or an int vocab size."""
    shards, params = load_meta_shards(ckpt_dir, verbose)
    vocab = tokenizer if isinstance(tokenizer, int) else len(tokenizer)
    config = config_from_params_json(params, vocab, max_seq_len, strict=strict)
    sd = merge_meta_shards(shards, config.num_hidden_layers, dtype)
    return meta_state_dict_to_params(sd, config.num_hidden_layers), config


# ----------------------------------------------------------------------------------
# Fake checkpoints (tests / synthetic runs)
# ----------------------------------------------------------------------------------
def random_meta_state_dict(config: LLaMAConfig, seed: int = 0, std: float = 0.02,
                           dtype=torch.bfloat16, norm_jitter: float = 0.1) -> Dict[str, torch.Tensor]:
    """Random Meta-layout weights (norm scales ~1 with jitter so folding is exercised)."""
    g = torch.Generator().manual_seed(seed)
    c = config
    d, hd, f, v = c.hidden_size, c.head_dim, c.intermediate_size, c.vocab_size
    hq, hkv = c.num_attention_heads * hd, c.num_key_value_heads * hd

    def rnd(*shape, s=std):
        return (torch.randn(*shape, generator=g) * s).to(dtype)

    def norm():
        return (1.0 + norm_jitter * torch.randn(d, generator=g)).to(dtype)

    sd = {"tok_embeddings.weight": rnd(v, d, s=1.0), "norm.weight": norm(), "output.weight": rnd(v, d)}
    for i in range(c.num_hidden_layers):
        pre = f"layers.{i}."
        sd[pre + "attention.wq.weight"] = rnd(hq, d)
        sd[pre + "attention.wk.weight"] = rnd(hkv, d)
        sd[pre + "attention.wv.weight"] = rnd(hkv, d)
        sd[pre + "attention.wo.weight"] = rnd(d, hq)
        sd[pre + "feed_forward.w1.weight"] = rnd(f, d)
        sd[pre + "feed_forward.w2.weight"] = rnd(d, f)
        sd[pre + "feed_forward.w3.weight"] = rnd(f, d)
        sd[pre + "attention_norm.weight"] = norm()
        sd[pre + "ffn_norm.weight"] = norm()
    return sd


def params_json_for(config: LLaMAConfig, multiple_of: int, ffn_dim_multiplier=None) -> Dict:
    p = {"dim": config.hidden_size, "n_layers": config.num_hidden_layers, "n_heads": config.num_attention_heads,
         "multiple_of": multiple_of, "norm_eps": config.rms_norm_eps, "vocab_size": -1}
    if config.num_key_value_heads != config.num_attention_heads:
        p["n_kv_heads"] = config.num_key_value_heads
    if ffn_dim_multiplier is not None:
        p["ffn_dim_multiplier"] = ffn_dim_multiplier
    if config.rope_theta != 10000.0:
        p["rope_theta"] = config.rope_theta
    return p


def save_meta_checkpoint(sd: Dict[str, torch.Tensor], params_json: Dict, out_dir: str, n_shards: int = 1,
                         vocab_parallel_embedding: bool = False) -> None:
    """Write ``consolidated.XX.pth`` + ``params.json`` split like Meta's MP checkpoints
    (``download.sh``: 7B/13B/30B/65B = 1/2/4/8 shards). ``vocab_parallel_embedding``
    selects the Llama-3 embedding split (vocab) instead of LLaMA-1/2 (model dim)."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "params.json"), "w") as f:
        json.dump(params_json, f)
    for r in range(n_shards):
        shard = {}
        for k, t in sd.items():
            if k == "tok_embeddings.weight":
                ax = 0 if vocab_parallel_embedding else 1
            elif k == "output.weight" or any(k.endswith(c + ".weight") for c in _COL):
                ax = 0
            elif any(k.endswith(c + ".weight") for c in _ROW):
                ax = 1
            else:
                shard[k] = t.clone()
                continue
            shard[k] = t.chunk(n_shards, ax)[r].clone()
        torch.save(shard, os.path.join(out_dir, f"consolidated.{r:02d}.pth"))


# ----------------------------------------------------------------------------------
# Per-rank loading (tensor parallel, one process per GPU)
# ----------------------------------------------------------------------------------
def _global_slice(pieces: List[torch.Tensor], cat_axis: int, axis: int, lo: int, hi: int) -> torch.Tensor:
    """Rows/cols [lo, hi) along ``axis`` of ``cat(pieces, cat_axis)`` without materialising the
    concatenation (pieces are mmapped Meta shards)."""
    if len(pieces) == 1:
        return pieces[0].narrow(axis, lo, hi - lo)
    if axis != cat_axis:
        return torch.cat([p.narrow(axis, lo, hi - lo) for p in pieces], cat_axis)
    out, start = [], 0
    for p in pieces:
        n = p.shape[axis]
        a, b = max(lo, start), min(hi, start + n)
        if a < b:
            out.append(p.narrow(axis, a - start, b - a))
        start += n
    return out[0] if len(out) == 1 else torch.cat(out, axis)


def load_meta_rank(ckpt_dir: str, tokenizer, rank: int, size: int, max_seq_len: int = 2048,
                   dtype: Optional[torch.dtype] = torch.bfloat16, verbose: bool = False):
    """This TP rank's parameters straight from Meta ``consolidated.XX.pth`` shards.

    Each tensor is read as the slices the rank needs (Megatron split of ``partition.py:62-78``:
    wq/wk/wv/w1/w3/output column-parallel, wo/w2 row-parallel, embedding and norms replicated)
    from the mmapped shards, whatever the checkpoint's own MP degree -- so 8 ranks loading a
    70B model touch ~1/8 of the bytes each instead of 8 full host copies (the reference merges
    everything to fp32 on the host first, convert_weights.py:66-89). Returns
    ``(params, config)`` with ``params`` ready for ``model.load_params(params, sharded=True)``."""
    shards, params_json = load_meta_shards(ckpt_dir, verbose)
    vocab = tokenizer if isinstance(tokenizer, int) else len(tokenizer)
    config = config_from_params_json(params_json, vocab, max_seq_len)
    n = len(shards)
    emb = [s["tok_embeddings.weight"] for s in shards]
    if n > 1:
        d_s, v_s = emb[0].shape[1], emb[0].shape[0]
        emb_axis = 1 if all(e.shape[0] == v_s for e in emb) and shards[0]["norm.weight"].shape[0] == d_s * n else 0
    else:
        emb_axis = 0

    def cvt(t):
        return t.contiguous() if dtype is None else t.to(dtype).contiguous()

    def col(key):  # [out, in] split on out
        pieces = [s[key] for s in shards]
        total = sum(p.shape[0] for p in pieces)
        c = total // size
        return cvt(_global_slice(pieces, 0, 0, rank * c, (rank + 1) * c))

    def row(key):  # [out, in] split on in
        pieces = [s[key] for s in shards]
        total = sum(p.shape[1] for p in pieces)
        c = total // size
        return cvt(_global_slice(pieces, 1, 1, rank * c, (rank + 1) * c))

    sd = {"tok_embeddings.weight": cvt(_cat(emb, emb_axis, None)),
          "norm.weight": cvt(shards[0]["norm.weight"]),
          "output.weight": col("output.weight")}
    for i in range(config.num_hidden_layers):
        pre = f"layers.{i}."
        for name in _COL:
            sd[pre + name + ".weight"] = col(pre + name + ".weight")
        for name in _ROW:
            sd[pre + name + ".weight"] = row(pre + name + ".weight")
        for name in ("attention_norm", "ffn_norm"):
            sd[pre + name + ".weight"] = cvt(shards[0][pre + name + ".weight"])
    return meta_state_dict_to_params(sd, config.num_hidden_layers), config
