"""Model configuration.

Parity with the reference:
  * ``LLaMAConfig`` mirrors ``jax_llama/config.py:70-116`` (same field names and
    defaults: the 7B shape, ``num_key_value_heads`` defaulting to
    ``num_attention_heads``, dropouts 0, ``rope_theta`` 1e4).
  * ``ModelArgs`` / ``config_from_params`` mirror ``jax_llama/convert_weights.py:13-50``
    (Meta ``params.json`` -> config, including the SwiGLU hidden-size formula).

Unlike the reference we do not subclass ``transformers.PretrainedConfig`` (importing
transformers costs seconds and drags in an unrelated framework); the class offers the
subset of that API the reference relies on (``to_dict``/``from_dict``/
``save_pretrained``/``from_pretrained``, ``return_dict``/``output_*`` flags).
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass
from typing import Any, Dict, Optional


class LLaMAConfig:
    """Architecture hyper-parameters of a LLaMA-1/2/3 decoder (reference ``config.py:70``)."""

    model_type = "llama"

    def __init__(
        self,
        vocab_size: int = 32000,
        hidden_size: int = 4096,
        intermediate_size: int = 11008,
        num_hidden_layers: int = 32,
        num_attention_heads: int = 32,
        num_key_value_heads: Optional[int] = None,
        max_sequence_length: int = 2048,
        rms_norm_eps: float = 1e-6,
        initializer_range: float = 0.02,
        use_cache: bool = True,
        pad_token_id: int = -1,
        bos_token_id: int = 1,
        eos_token_id: int = 2,
        resid_pdrop: float = 0.0,
        embd_pdrop: float = 0.0,
        attn_pdrop: float = 0.0,
        tie_word_embeddings: bool = False,
        gradient_checkpointing: bool = False,
        rope_theta: float = 10000.0,
        output_attentions: bool = False,
        output_hidden_states: bool = False,
        return_dict: bool = True,
        **kwargs: Any,
    ):
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.initializer_range = initializer_range
        self.intermediate_size = intermediate_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        if num_key_value_heads is None:
            num_key_value_heads = num_attention_heads
        self.num_key_value_heads = num_key_value_heads
        self.max_sequence_length = max_sequence_length
        self.rms_norm_eps = rms_norm_eps
        self.use_cache = use_cache
        self.pad_token_id = pad_token_id
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.resid_pdrop = resid_pdrop
        self.embd_pdrop = embd_pdrop
        self.attn_pdrop = attn_pdrop
        self.tie_word_embeddings = tie_word_embeddings
        self.gradient_checkpointing = gradient_checkpointing
        self.rope_theta = rope_theta
        self.output_attentions = output_attentions
        self.output_hidden_states = output_hidden_states
        self.return_dict = return_dict
        # Unknown keys are kept (HF PretrainedConfig behaviour) so configs round-trip.
        for k, v in kwargs.items():
            setattr(self, k, v)
        if self.hidden_size % self.num_attention_heads:
            raise ValueError("hidden_size must be divisible by num_attention_heads")
        if self.num_attention_heads % self.num_key_value_heads:
            raise ValueError("num_attention_heads must be divisible by num_key_value_heads")

    # ---- derived -------------------------------------------------------------------
    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def num_key_value_groups(self) -> int:
        return self.num_attention_heads // self.num_key_value_heads

    def num_parameters(self) -> int:
        d, f, v, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        kv = self.num_key_value_heads * self.head_dim
        per_layer = d * d * 2 + d * kv * 2 + 3 * d * f + 2 * d
        head = 0 if self.tie_word_embeddings else v * d
        return v * d + L * per_layer + d + head

    # ---- (de)serialisation ---------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        out = dict(self.__dict__)
        out["model_type"] = self.model_type
        return out

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "LLaMAConfig":
        d = dict(d)
        d.pop("model_type", None)
        return cls(**d)

    def to_json_string(self) -> str:
        return json.dumps(self.to_dict(), indent=2, sort_keys=True)

    def save_pretrained(self, save_directory: str) -> None:
        os.makedirs(save_directory, exist_ok=True)
        with open(os.path.join(save_directory, "config.json"), "w") as f:
            f.write(self.to_json_string())

    @classmethod
    def from_pretrained(cls, path: str) -> "LLaMAConfig":
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def __eq__(self, other: object) -> bool:
        return isinstance(other, LLaMAConfig) and self.to_dict() == other.to_dict()

    def __repr__(self) -> str:
        return f"LLaMAConfig {self.to_json_string()}"


# -------------------------------------------------------------------------------------
# Meta params.json handling (reference convert_weights.py:13-50)
# -------------------------------------------------------------------------------------
@dataclass
class ModelArgs:
    """Meta ``params.json`` schema. Constructing with unknown keys raises ``TypeError``
    exactly like the reference (``convert_weights.py:91``); ``from_params_json`` offers a
    tolerant path that also understands Llama-3.1 ``use_scaled_rope``."""

    dim: int = 512
    n_layers: int = 8
    n_heads: int = 8
    n_kv_heads: Optional[int] = None
    vocab_size: int = -1
    multiple_of: int = 256
    ffn_dim_multiplier: Optional[float] = None
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    max_batch_size: int = 32
    max_seq_len: int = 2048

    @classmethod
    def from_params_json(cls, params: Dict[str, Any], strict: bool = True) -> "ModelArgs":
        if strict:
            return cls(**params)
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in params.items() if k in names})


def swiglu_hidden_size(dim: int, multiple_of: int, ffn_dim_multiplier: Optional[float] = None) -> int:
    """FFN width rule of Meta's FeedForward (reference ``convert_weights.py:36-39``)."""
    hidden = int(2 * (dim * 4) / 3)
    if ffn_dim_multiplier is not None:
        hidden = int(ffn_dim_multiplier * hidden)
    return multiple_of * ((hidden + multiple_of - 1) // multiple_of)


def config_from_params(args: ModelArgs) -> LLaMAConfig:
    return LLaMAConfig(
        vocab_size=args.vocab_size,
        hidden_size=args.dim,
        intermediate_size=swiglu_hidden_size(args.dim, args.multiple_of, args.ffn_dim_multiplier),
        num_hidden_layers=args.n_layers,
        num_attention_heads=args.n_heads,
        num_key_value_heads=args.n_kv_heads,
        max_sequence_length=args.max_seq_len,
        rms_norm_eps=args.norm_eps,
        rope_theta=args.rope_theta,
    )


# -------------------------------------------------------------------------------------
# Named presets (Meta params.json values; MODEL_CARD.md:82-91 for LLaMA-1 shapes).
# Used by the synthetic/random-init paths (bench.py, examples --synthetic).
# -------------------------------------------------------------------------------------
_META_PARAMS: Dict[str, Dict[str, Any]] = {
    "llama1-7b": dict(dim=4096, n_layers=32, n_heads=32, multiple_of=256, norm_eps=1e-6, vocab_size=32000),
    "llama1-13b": dict(dim=5120, n_layers=40, n_heads=40, multiple_of=256, norm_eps=1e-6, vocab_size=32000),
    "llama1-33b": dict(dim=6656, n_layers=60, n_heads=52, multiple_of=256, norm_eps=1e-6, vocab_size=32000),
    "llama1-65b": dict(dim=8192, n_layers=80, n_heads=64, multiple_of=256, norm_eps=1e-5, vocab_size=32000),
    "llama2-7b": dict(dim=4096, n_layers=32, n_heads=32, multiple_of=256, norm_eps=1e-5, vocab_size=32000),
    "llama2-13b": dict(dim=5120, n_layers=40, n_heads=40, multiple_of=256, norm_eps=1e-5, vocab_size=32000),
    "llama2-70b": dict(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, multiple_of=4096,
                       ffn_dim_multiplier=1.3, norm_eps=1e-5, vocab_size=32000),
    "llama3-8b": dict(dim=4096, n_layers=32, n_heads=32, n_kv_heads=8, multiple_of=1024,
                      ffn_dim_multiplier=1.3, norm_eps=1e-5, rope_theta=500000.0, vocab_size=128256),
    "llama3-70b": dict(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, multiple_of=4096,
                       ffn_dim_multiplier=1.3, norm_eps=1e-5, rope_theta=500000.0, vocab_size=128256),
    # The tiny fixture of jax_test.py:28-41 (dim 32, 4 layers, 4 heads, 2 kv heads, vocab 256).
    "tiny": dict(dim=32, n_layers=4, n_heads=4, n_kv_heads=2, multiple_of=2, norm_eps=1e-5,
                 vocab_size=256, max_seq_len=64),
}
_ALIASES = {"7b": "llama2-7b", "8b": "llama3-8b", "13b": "llama2-13b", "33b": "llama1-33b",
            "65b": "llama1-65b", "70b": "llama3-70b"}


def preset_names():
    return sorted(_META_PARAMS)


def get_preset(name: str, max_seq_len: Optional[int] = None, **overrides: Any) -> LLaMAConfig:
    name = _ALIASES.get(name.lower(), name.lower())
    if name not in _META_PARAMS:
        raise KeyError(f"unknown model preset {name!r}; known: {preset_names()}")
    p = dict(_META_PARAMS[name])
    if max_seq_len is not None:
        p["max_seq_len"] = max_seq_len
    cfg = config_from_params(ModelArgs(**p))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg
