"""jax_llama_amd — an MI355X-native (gfx950 / CDNA4) LLaMA-1/2/3 inference framework with the
public API of LSaldyt/JAX_llama (reference ``jax_llama/__init__.py:4-10``).

Framework layer: PyTorch-ROCm. Hot path: hand-written HIP kernels (``csrc/kernels``).
Multi-GPU: one process per GPU, RCCL + a custom xGMI all-reduce. Decode: hipGraph replay.
"""
from .config import LLaMAConfig, ModelArgs, config_from_params, get_preset, swiglu_hidden_size
from .generation import LLaMA
from .models import (CausalLMOutput, FlaxLLaMAForCausalLM, FlaxLLaMAModel, KVCache, LLaMAForCausalLM,
                     LLaMAModel)
from .parallel.partition import (Mesh, P, PartitionSpec, get_llama_param_partition_spec,
                                 with_named_sharding_constraint, with_sharding_constraint)
from .runtime.engine import GenerationConfig
from .tokenizer import ChatFormat, LLaMA2Tokenizer, LLaMA3Tokenizer
from .utils.checkpoint import convert_llama_weights

__version__ = "0.1.0"

__all__ = [
    "LLaMAConfig", "ModelArgs", "config_from_params", "get_preset", "swiglu_hidden_size",
    "LLaMA", "LLaMAForCausalLM", "LLaMAModel", "FlaxLLaMAForCausalLM", "FlaxLLaMAModel",
    "CausalLMOutput", "KVCache", "GenerationConfig",
    "Mesh", "P", "PartitionSpec", "get_llama_param_partition_spec", "with_named_sharding_constraint",
    "with_sharding_constraint", "LLaMA2Tokenizer", "LLaMA3Tokenizer", "ChatFormat", "convert_llama_weights",
]
