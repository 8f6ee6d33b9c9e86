"""LLaMA-1/2/3 causal LM (inference) on the MI355X op layer.

Reference structure (``/root/reference/jax_llama/model.py``):
  * ``FlaxLLaMAAttention`` (:105-300), ``FlaxLLaMAMLP`` (:302-340), ``FlaxLLaMABlock``
    (:342-400), ``FlaxLLaMABlockCollection`` (:548-600), ``FlaxLLaMAModule`` (:602-677),
    ``FlaxLLaMAForCausalLMModule`` (:691-741), HF wrapper ``FlaxLLaMAPreTrainedModel``
    (:402-546) and the generation adapters (:744-772).

MI355X design (not a translation):
  * one fused op per projection: RMSNorm is folded into the following GEMM
    (``inv_rms`` applied in the epilogue), ``wq|wk|wv`` are one GEMM, ``w1|w3`` one GEMM
    with a SiLU*mul epilogue, ``wo``/``w2`` accumulate straight into the fp32 residual
    stream (``ops.linear_residual``);
  * RoPE (interleaved pairs, Meta layout) + KV-cache write is one kernel; attention reads
    the ``[B, Hkv, T, Dh]`` cache directly with GQA indexing (no ``repeat_kv`` copy) and
    builds the causal/padding mask in-kernel from ``(slot, kv_start)`` — nothing like the
    reference's materialised ``(L, L)`` mask;
  * logits are computed for the last position only during generation;
  * tensor parallelism is explicit SPMD: column-parallel qkv/w1|w3, row-parallel wo/w2
    followed by an all-reduce, vocab-parallel lm_head (``parallel/partition.py`` rules).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..config import LLaMAConfig
from ..ops import reference as ref
from ..parallel.comm import NO_COMM, TPComm
from ..parallel.partition import shard_tree
from .kv_cache import KVCache
from .modules import LLaMABlockCollection
from .weights import PackedLinear

BF16 = torch.bfloat16


def _t(x) -> torch.Tensor:
    if torch.is_tensor(x):
        return x
    return torch.as_tensor(np.asarray(x))


@dataclass
class CausalLMOutput:
    """Mirror of HF ``FlaxCausalLMOutput`` (+ ``past_key_values``) with dict-style access."""

    logits: Optional[torch.Tensor] = None
    past_key_values: Optional[KVCache] = None
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None
    attentions: Optional[Tuple[torch.Tensor, ...]] = None

    def __getitem__(self, k):
        if isinstance(k, int):
            return self.to_tuple()[k]
        return getattr(self, k)

    def __setitem__(self, k, v):
        setattr(self, k, v)

    def to_tuple(self):
        return tuple(v for v in (self.logits, self.past_key_values, self.hidden_states, self.attentions)
                     if v is not None)


@dataclass
class BaseModelOutput:
    last_hidden_state: torch.Tensor = None
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None
    attentions: Optional[Tuple[torch.Tensor, ...]] = None

    def __getitem__(self, k):
        if isinstance(k, int):
            return tuple(v for v in (self.last_hidden_state, self.hidden_states, self.attentions)
                         if v is not None)[k]
        return getattr(self, k)


class LayerWeights:
    __slots__ = ("qkv", "o", "gu", "down", "attention_norm", "ffn_norm")

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)


def mask_to_kv_start(mask: torch.Tensor, device) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Turn a (B, T) 0/1 key mask into ``kv_start`` (first valid slot per row) when every
    row is of the left-padded form ``0...0 1...1``; otherwise also return the mask itself
    (uint8, on ``device``) for the kernels' general masked path."""
    m = mask.detach().to("cpu").to(torch.int64)
    b, t = m.shape
    valid = m != 0
    first = torch.where(valid.any(1), valid.to(torch.int8).argmax(1), torch.full((b,), t, dtype=torch.int64))
    after = torch.arange(t)[None, :] >= first[:, None]
    if bool((after & ~valid).any()):  # a hole after the first valid key: general masked path
        return torch.zeros(b, dtype=torch.int32, device=device), m.to(torch.uint8).to(device).contiguous()
    return first.to(torch.int32).to(device), None


_DTYPE_NAMES = {"float32": torch.float32, "fp32": torch.float32, "f32": torch.float32,
                "bfloat16": BF16, "bf16": BF16}


def _resolve_dtype(d, default):
    """torch dtype, a name, or a numpy / jnp-style dtype object (``jnp.float32``) -> torch dtype."""
    if d is None:
        return default
    if isinstance(d, torch.dtype):
        return d
    name = d if isinstance(d, str) else getattr(d, "__name__", None) or getattr(d, "name", None) or str(d)
    name = str(name).split(".")[-1].strip("'>")
    if name not in _DTYPE_NAMES:
        raise ValueError(f"unsupported dtype {d!r}")
    return _DTYPE_NAMES[name]


def _resolve_precision(p) -> str:
    """jax.lax.Precision-like values -> 'default' | 'highest'."""
    if p is None:
        return "default"
    name = str(getattr(p, "name", p)).lower().split(".")[-1]
    if name in ("default", "fastest", "bfloat16"):
        return "default"
    if name in ("highest", "float32", "high", "tensorfloat32"):
        return "highest"
    raise ValueError(f"unsupported precision {p!r}")


class LLaMAForCausalLM:
    """Causal LM with an HF-flavoured call API (reference ``FlaxLLaMAForCausalLM``)."""

    base_model_prefix = "transformer"
    config_class = LLaMAConfig

    def __init__(self, config: LLaMAConfig, input_shape: Tuple[int, ...] = (1, 1), seed: int = 0, dtype=None,
                 _do_init: bool = True, precision=None, param_dtype=None, device="cpu",
                 comm: Optional[TPComm] = None, rope_length: Optional[int] = None, **kwargs):
        """Reference ``FlaxLLaMAPreTrainedModel.__init__(config, input_shape, seed, dtype, _do_init,
        **kwargs)`` (``model.py:412-422``) with the module kwargs ``param_dtype`` / ``precision``
        (``model.py:107-109``; ``jax_test.py:433`` passes ``precision='highest'``).

        * ``_do_init=True`` (HF default): random-initialise the weights (``init_weights(seed)``);
          ``_do_init=False`` (``jax_example.py:29``): weights come later (``load_params`` / ``params=``).
        * ``dtype``: dtype of returned activations/logits. The MFMA kernels always run bf16 operands
          with fp32 accumulation; ``float32`` (the reference default) and ``bfloat16`` are accepted.
        * ``param_dtype``: storage dtype of the weights — bf16 (the MFMA operand); fp32 is accepted and
          converted (the reference converts every checkpoint to fp32, ``convert_weights.py:68-88``).
        * ``precision``: ``None``/``'default'``, or ``'highest'``/``'float32'``, which (as in the
          reference, where only ``lm_head`` honours it, ``model.py:698``) computes the logits with fp32
          lm_head weights and an fp32 GEMM."""
        if kwargs:
            unknown = sorted(kwargs)
            raise TypeError(f"unexpected model kwargs {unknown}")
        self.dtype = _resolve_dtype(dtype, torch.float32)
        if self.dtype not in (torch.float32, BF16):
            raise ValueError(f"dtype must be float32 or bfloat16, got {dtype}")
        pd = _resolve_dtype(param_dtype, BF16)
        if pd not in (torch.float32, BF16):
            raise ValueError(f"param_dtype must be float32 or bfloat16, got {param_dtype}")
        self.param_dtype = BF16  # MFMA operand dtype (fp32 parameters are converted on load)
        self.precision = _resolve_precision(precision)
        self.input_shape = tuple(input_shape)
        self.seed = int(seed)
        self._missing_keys = set()
        self.config = config
        self.device = torch.device(device)
        self.comm = comm or NO_COMM
        tp = self.comm.size
        c = config
        for name, val in (("num_attention_heads", c.num_attention_heads),
                          ("num_key_value_heads", c.num_key_value_heads),
                          ("intermediate_size", c.intermediate_size), ("vocab_size", c.vocab_size)):
            if val % tp:
                raise ValueError(f"{name}={val} is not divisible by tensor-parallel degree {tp}")
        self.n_heads = c.num_attention_heads // tp
        self.n_kv_heads = c.num_key_value_heads // tp
        self.head_dim = c.head_dim
        self.ffn = c.intermediate_size // tp
        self.vocab_local = c.vocab_size // tp
        self.eps = float(c.rms_norm_eps)
        # RoPE table over 2 * max_sequence_length positions (reference model.py:156-161), fp32.
        self.rope_length = rope_length or 2 * c.max_sequence_length
        self.rope = ref.rope_table(self.head_dim, self.rope_length, c.rope_theta,
                                   scaled=bool(getattr(c, "use_scaled_rope", False))).to(self.device)
        self.wte: Optional[torch.Tensor] = None
        self.ln_f: Optional[torch.Tensor] = None
        self.lm_head: Optional[PackedLinear] = None
        self.layers: List[LayerWeights] = [LayerWeights() for _ in range(c.num_hidden_layers)]
        self.blocks = LLaMABlockCollection(self)  # reference FlaxLLaMABlockCollection (model.py:548)
        self._params_id = None
        self.lm_head_f32: Optional[torch.Tensor] = None  # [V/tp, D] fp32 (precision='highest')
        if _do_init:
            self.init_random(seed=self.seed)

    # ------------------------------------------------------------------ weights
    @property
    def tp_rank(self):
        return self.comm.rank

    @property
    def tp_size(self):
        return self.comm.size

    def load_params(self, params: Dict[str, Any], sharded: bool = False) -> "LLaMAForCausalLM":
        """Load a reference-named parameter tree (Flax ``(in, out)`` kernel orientation, as
        returned by ``convert_llama_weights``). ``sharded=False``: the tree is the full
        model and this rank keeps its TP shard (partition rules of ``partition.py``)."""
        if not sharded:
            params = shard_tree(params, self.tp_rank, self.tp_size)
        dev = self.device
        tr = params["transformer"]
        self.wte = _t(tr["wte"]["embedding"]).to(dev, BF16).contiguous()
        self.ln_f = _t(tr["ln_f"]["kernel"]).to(dev, torch.float32)
        for i, lw in enumerate(self.layers):
            blk = tr["h"][str(i)]
            att, ff = blk["attention"], blk["feed_forward"]
            wq = _t(att["wq"]["kernel"]).t()
            wk = _t(att["wk"]["kernel"]).t()
            wv = _t(att["wv"]["kernel"]).t()
            lw.attention_norm = _t(blk["attention_norm"]["kernel"]).to(dev, torch.float32)
            lw.ffn_norm = _t(blk["ffn_norm"]["kernel"]).to(dev, torch.float32)
            lw.qkv = PackedLinear.from_dense(torch.cat([wq, wk, wv], 0), dev, fold=lw.attention_norm)
            lw.o = PackedLinear.from_dense(_t(att["wo"]["kernel"]).t(), dev)
            gu = ref.interleave_gate_up(_t(ff["w1"]["kernel"]).t(), _t(ff["w3"]["kernel"]).t())
            lw.gu = PackedLinear.from_dense(gu, dev, fold=lw.ffn_norm)
            lw.down = PackedLinear.from_dense(_t(ff["w2"]["kernel"]).t(), dev)
        if self.config.tie_word_embeddings:
            full = _t(tr["wte"]["embedding"])
            lm = full.narrow(0, self.tp_rank * self.vocab_local, self.vocab_local)
        else:
            lm = _t(params["lm_head"]["kernel"]).t()
        self.lm_head = PackedLinear.from_dense(lm, dev, fold=self.ln_f)
        self.lm_head_f32 = _t(lm).to(dev, torch.float32).contiguous() if self.precision == "highest" else None
        self._params_id = id(params)
        return self

    def init_random(self, seed: int = 0, std: Optional[float] = None) -> "LLaMAForCausalLM":
        """Random-init every weight directly in the device layout (synthetic benchmarks).
        Norm weights are ones (folded), like Flax's RMSNorm init."""
        c = self.config
        std = c.initializer_range if std is None else std
        dev = self.device
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed + 1000 * self.tp_rank)
        d, hd = c.hidden_size, self.head_dim
        self.wte = torch.empty(c.vocab_size, d, dtype=BF16, device=dev)
        # embedding rows identical on every TP rank
        g0 = torch.Generator(device=dev)
        g0.manual_seed(seed)
        self.wte.normal_(0.0, 1.0, generator=g0)
        self.ln_f = torch.ones(d, dtype=torch.float32, device=dev)
        nqkv = (self.n_heads + 2 * self.n_kv_heads) * hd
        for lw in self.layers:
            lw.attention_norm = torch.ones(d, dtype=torch.float32, device=dev)
            lw.ffn_norm = torch.ones(d, dtype=torch.float32, device=dev)
            lw.qkv = PackedLinear.random(nqkv, d, dev, std, gen)
            lw.o = PackedLinear.random(d, self.n_heads * hd, dev, std, gen)
            lw.gu = PackedLinear.random(2 * self.ffn, d, dev, std, gen)
            lw.down = PackedLinear.random(d, self.ffn, dev, std, gen)
        self.lm_head = PackedLinear.random(self.vocab_local, d, dev, std, gen)
        self.lm_head_f32 = self.lm_head.dense().float().contiguous() if self.precision == "highest" else None
        return self

    def init_weights(self, rng=None, input_shape: Optional[Tuple[int, ...]] = None, params: Optional[Dict] = None,
                     std: Optional[float] = None) -> Dict:
        """Reference ``init_weights(rng, input_shape, params=None)`` (``model.py:424-457``): a random
        parameter tree with the reference names and Flax ``(in, out)`` kernel layout (fp32, host). With
        ``params`` given, every key it lacks (``self._missing_keys``, or any absent leaf) is filled from
        the random tree and the completed tree is returned. ``rng``: int seed, torch.Generator or a
        PRNG-key-like integer array."""
        from ..parallel.partition import flatten_tree, unflatten_tree
        from ..utils.checkpoint import meta_state_dict_to_params, random_meta_state_dict
        if rng is None:
            seed = self.seed
        elif isinstance(rng, torch.Generator):
            seed = int(rng.initial_seed())
        else:
            seed = int(np.asarray(rng).reshape(-1)[-1])
        c = self.config
        sd = random_meta_state_dict(c, seed=seed, std=c.initializer_range if std is None else std,
                                    dtype=torch.float32, norm_jitter=0.0)
        rand = meta_state_dict_to_params(sd, c.num_hidden_layers)
        if c.tie_word_embeddings:
            rand.pop("lm_head", None)
        if params is None:
            return rand
        flat_r, flat_p = flatten_tree(rand), flatten_tree(params)
        missing = set(self._missing_keys) | (set(flat_r) - set(flat_p))
        for k in missing:
            flat_p[k] = flat_r[k]
        self._missing_keys = set()
        return unflatten_tree(flat_p)

    def save_pretrained(self, save_directory: str) -> str:
        """Deployed-form safetensors checkpoint of this rank (``utils/native_ckpt.py``)."""
        from ..utils.native_ckpt import save_pretrained
        return save_pretrained(self, save_directory)

    @classmethod
    def from_pretrained(cls, directory: str, device="cpu", comm: Optional[TPComm] = None):
        """Reload a ``save_pretrained`` checkpoint (same TP degree) straight into the kernel layout."""
        from ..utils.native_ckpt import from_pretrained
        return from_pretrained(directory, device=device, comm=comm)

    def weight_bytes(self) -> int:
        n = self.wte.numel() * 2 + self.lm_head.nbytes()
        for lw in self.layers:
            n += lw.qkv.nbytes() + lw.o.nbytes() + lw.gu.nbytes() + lw.down.nbytes()
        return n

    def streamed_weight_bytes_per_token(self) -> int:
        """Bytes of weights read per decode step (embedding rows excluded)."""
        return self.weight_bytes() - self.wte.numel() * 2

    # ------------------------------------------------------------------ cache
    def init_cache(self, batch_size: int, max_length: int) -> KVCache:
        """Reference ``init_cache(B, T)`` (``model.py:459-476``) without a dummy forward."""
        if max_length > self.rope_length:
            raise ValueError(f"max_length {max_length} exceeds the RoPE table ({self.rope_length}); "
                             "raise config.max_sequence_length")
        return KVCache(self.config.num_hidden_layers, batch_size, self.n_kv_heads, max_length,
                       self.head_dim, self.device)

    # ------------------------------------------------------------------ core forward
    def _row_parallel(self, x: torch.Tensor, w: PackedLinear, h: torch.Tensor, hb: torch.Tensor,
                      x_packed: Optional[torch.Tensor] = None, mirror_packed: Optional[torch.Tensor] = None) -> None:
        """``h += x @ W^T`` where W is row-sharded. TP=1: the GEMM epilogue adds into the fp32 residual
        ``h`` and writes its bf16 mirror ``hb`` (the A operand of the next projection). TP>1: the GEMM
        writes only this rank's partial (``comm.reduce_dtype``, bf16 by default). Decode-sized partials: one
        custom collective kernel (or the GEMV itself, ``comm.FUSED``) sums them in fp32 in rank order, adds them to
        ``h`` and rewrites ``hb``. Prefill-sized partials: the GEMM writes them in fp32 (``comm.partial_dtype``) and RCCL
        sums them (RCCL's order; bf16 on the wire only with ``JLA_TP_RCCL_BF16=1``), then one kernel adds into ``h`` (``comm.all_reduce_residual_``;
        reference ``partition.py:67,70``)."""
        if self.comm.size == 1:
            ops.linear_residual(x, w, h, mirror=hb, x_packed=x_packed, mirror_packed=mirror_packed)
        elif self.comm.linear_residual_(x, w, h, hb, x_packed=x_packed, hb_pack=mirror_packed):
            pass  # decode: the GEMV exchanged its partials itself (one kernel; comm.FUSED)
        else:
            dt = self.comm.partial_dtype(x.numel() // x.shape[-1] * w.n, x.is_cuda)
            part = ops.linear(x, w, out_dtype=dt, x_packed=x_packed)
            self.comm.all_reduce_residual_(part, h, hb, hb_pack=mirror_packed, owned=True)

    def forward_tokens(self, ids: torch.Tensor, positions: torch.Tensor, cache: KVCache, slot0,
                       kv_start: torch.Tensor, key_mask: Optional[torch.Tensor] = None,
                       logits_mode: str = "last", collect_hidden: bool = False,
                       collect_attn: bool = False):
        """Run all layers for ``ids [B, S]`` placed at cache slots ``slot0 .. slot0+S-1``.

        ``slot0``: int or device int32[1] tensor (graph capture). Returns
        ``(logits_local, h, hidden_states, attentions)`` where logits are this rank's
        vocab shard: ``[B, V/tp]`` ("last"), ``[B*S, V/tp]`` ("all"), None ("none"), or the
        shard's greedy ``(idx int32[B], val fp32[B])`` of the last position ("argmax")."""
        with ops.autotune.tp_scope(self.comm):  # TP: rank 0 picks the kernel plans for every rank
            return self._forward_tokens(ids, positions, cache, slot0, kv_start, key_mask, logits_mode,
                                        collect_hidden, collect_attn)

    def _forward_tokens(self, ids, positions, cache, slot0, kv_start, key_mask, logits_mode, collect_hidden,
                        collect_attn):
        b, s = ids.shape
        d = self.config.hidden_size
        # residual stream: fp32 h plus its bf16 mirror hb (the A operand of every projection
        # that follows a norm; RMSNorm statistics are taken from these bf16 values)
        hb = torch.empty(b * s, d, dtype=BF16, device=self.device)
        h = ops.embedding(ids.reshape(-1), self.wte, mirror=hb)
        hidden, attns = self.blocks(h, hb, positions, cache, slot0, kv_start, key_mask, s,
                                    output_hidden_states=collect_hidden, output_attentions=collect_attn)
        if logits_mode == "none":
            logits = None
        elif self.precision == "highest":  # fp32 lm_head weights + fp32 GEMM (reference model.py:698-736)
            hl = h if logits_mode == "all" else h.reshape(b, s, d)[:, -1].contiguous()
            logits = ops.linear_f32(self.final_norm(hl), self.lm_head_f32)
            if logits_mode == "argmax":
                logits = ops.argmax(logits.contiguous())
        elif logits_mode == "argmax":  # greedy: (idx, val) of this rank's vocab shard, argmax fused in the GEMM
            logits = ops.linear_argmax(hb.reshape(b, s, d)[:, -1].contiguous(), self.lm_head, rms_eps=self.eps)
        else:
            hl = hb if logits_mode == "all" else hb.reshape(b, s, d)[:, -1].contiguous()
            logits = ops.linear(hl, self.lm_head, rms_eps=self.eps, out_dtype=torch.float32)
        return logits, h, hidden, attns

    def gather_logits(self, logits_local: torch.Tensor) -> torch.Tensor:
        """Vocab-parallel ``[M, V/tp]`` -> full ``[M, V]`` (all-gather over TP)."""
        if self.comm.size == 1:
            return logits_local
        g = self.comm.all_gather(logits_local)  # [tp, M, V/tp]
        return g.permute(1, 0, 2).reshape(logits_local.shape[0], -1)

    def final_norm(self, h: torch.Tensor) -> torch.Tensor:
        return ops.rmsnorm(h, self.ln_f, self.eps)

    # ------------------------------------------------------------------ HF-style API
    def _prepare_call(self, input_ids, attention_mask, position_ids, past_key_values):
        ids = _t(input_ids).to(self.device, torch.int32)
        b, s = ids.shape
        if position_ids is None:
            if past_key_values is not None:
                raise ValueError("Make sure to provide `position_ids` when passing `past_key_values`.")
            position_ids = torch.arange(s, dtype=torch.int32).expand(b, s)
        pos = _t(position_ids).to(self.device, torch.int32).reshape(b, s).contiguous()
        if past_key_values is None:
            cache = KVCache(self.config.num_hidden_layers, b, self.n_kv_heads, s, self.head_dim, self.device)
            slot0 = 0
        else:
            cache = past_key_values
            slot0 = cache.index
            if slot0 + s > cache.max_length:
                raise ValueError(f"cache overflow: {slot0}+{s} > {cache.max_length}")
        t_valid = slot0 + s
        if attention_mask is None:
            mask = torch.ones(b, t_valid, dtype=torch.int32)
        else:
            mask = _t(attention_mask).to("cpu").to(torch.int32)
            if mask.shape[1] >= t_valid:
                mask = mask[:, :t_valid]
            elif mask.shape[1] == s:
                mask = torch.cat([torch.ones(b, slot0, dtype=torch.int32), mask], 1)
            else:
                raise ValueError(f"attention_mask of shape {tuple(mask.shape)} does not cover {t_valid} slots")
        kv_start, key_mask = mask_to_kv_start(mask, self.device)
        return ids, pos, cache, slot0, kv_start, key_mask

    def __call__(self, input_ids, attention_mask=None, position_ids=None, params=None,
                 past_key_values: Optional[KVCache] = None, dropout_rng=None, train: bool = False,
                 output_attentions: Optional[bool] = None, output_hidden_states: Optional[bool] = None,
                 return_dict: Optional[bool] = None):
        """Reference ``FlaxLLaMAPreTrainedModel.__call__`` (``model.py:478-546``): logits for
        every position ``(B, S, V)`` fp32; the cache (if given) is updated in place and
        returned as ``past_key_values``."""
        if train:
            raise NotImplementedError("inference-only framework (reference dropout/remat paths are training-only)")
        if params is not None and id(params) != self._params_id:
            self.load_params(params)
        oa = self.config.output_attentions if output_attentions is None else output_attentions
        oh = self.config.output_hidden_states if output_hidden_states is None else output_hidden_states
        rd = self.config.return_dict if return_dict is None else return_dict
        ids, pos, cache, slot0, kv_start, key_mask = self._prepare_call(
            input_ids, attention_mask, position_ids, past_key_values)
        b, s = ids.shape
        logits, h, hidden, attns = self.forward_tokens(ids, pos, cache, slot0, kv_start, key_mask,
                                                       logits_mode="all", collect_hidden=oh,
                                                       collect_attn=oa)
        if past_key_values is not None:
            cache.advance(s)
        logits = self.gather_logits(logits).reshape(b, s, -1).to(self.dtype)
        hs = None
        if oh:
            hs = tuple(x.to(self.dtype) for x in hidden) + (self.final_norm(h).reshape(b, s, -1).to(self.dtype),)
        out = CausalLMOutput(logits=logits, past_key_values=past_key_values, hidden_states=hs,
                             attentions=tuple(attns) if oa else None)
        return out if rd else out.to_tuple()

    def prepare_inputs_for_generation(self, input_ids, max_length: int, attention_mask=None):
        """Reference ``model.py:748-767``: cache, extended (B, max_length) mask with the
        prompt mask written at (0, 0), and ``position_ids = cumsum(mask) - 1``."""
        ids = _t(input_ids)
        b, s = ids.shape
        cache = self.init_cache(b, max_length)
        ext = torch.ones(b, max_length, dtype=torch.int32)
        if attention_mask is not None:
            am = _t(attention_mask).to(torch.int32).cpu()
            position_ids = am.cumsum(-1) - 1
            ext[:, : am.shape[1]] = am
        else:
            position_ids = torch.arange(s, dtype=torch.int32).expand(b, s)
        return {"past_key_values": cache, "attention_mask": ext, "position_ids": position_ids}

    def update_inputs_for_generation(self, model_outputs, model_kwargs):
        """Reference ``model.py:769-772``."""
        model_kwargs["past_key_values"] = model_outputs.past_key_values
        model_kwargs["position_ids"] = _t(model_kwargs["position_ids"])[:, -1:] + 1
        return model_kwargs

    def generate(self, input_ids, attention_mask=None, generation_config=None, params=None,
                 prng_key=None, **kwargs):
        """HF ``generate`` equivalent (greedy / sampling with temperature, top-k, top-p),
        executed by the hipGraph decode engine (``runtime/engine.py``)."""
        from ..runtime.engine import generate as _generate
        if params is not None and id(params) != self._params_id:
            self.load_params(params)
        return _generate(self, input_ids, attention_mask, generation_config, prng_key=prng_key, **kwargs)


class LLaMAModel(LLaMAForCausalLM):
    """Backbone only (reference ``FlaxLLaMAModel``): returns the ``ln_f``-normalised hidden
    states instead of logits."""

    def __call__(self, input_ids, attention_mask=None, position_ids=None, params=None,
                 past_key_values: Optional[KVCache] = None, dropout_rng=None, train: bool = False,
                 output_attentions: Optional[bool] = None, output_hidden_states: Optional[bool] = None,
                 return_dict: Optional[bool] = None):
        if params is not None and id(params) != self._params_id:
            self.load_params(params)
        oa = self.config.output_attentions if output_attentions is None else output_attentions
        oh = self.config.output_hidden_states if output_hidden_states is None else output_hidden_states
        ids, pos, cache, slot0, kv_start, key_mask = self._prepare_call(
            input_ids, attention_mask, position_ids, past_key_values)
        b, s = ids.shape
        _, h, hidden, attns = self.forward_tokens(ids, pos, cache, slot0, kv_start, key_mask,
                                                  logits_mode="none", collect_hidden=oh, collect_attn=oa)
        if past_key_values is not None:
            cache.advance(s)
        last = self.final_norm(h).reshape(b, s, -1).to(self.dtype)
        return BaseModelOutput(last_hidden_state=last,
                               hidden_states=(tuple(x.to(self.dtype) for x in hidden) + (last,)) if oh else None,
                               attentions=tuple(attns) if oa else None)
