from .kv_cache import KVCache
from .llama import BaseModelOutput, CausalLMOutput, LLaMAForCausalLM, LLaMAModel, mask_to_kv_start
from .weights import PackedLinear

# Reference-compatible names (jax_llama/__init__.py:4)
FlaxLLaMAForCausalLM = LLaMAForCausalLM
FlaxLLaMAModel = LLaMAModel

__all__ = ["KVCache", "LLaMAForCausalLM", "LLaMAModel", "FlaxLLaMAForCausalLM", "FlaxLLaMAModel",
           "CausalLMOutput", "BaseModelOutput", "PackedLinear", "mask_to_kv_start"]
