from .kv_cache import KVCache
from .llama import BaseModelOutput, CausalLMOutput, LLaMAForCausalLM, LLaMAModel, mask_to_kv_start
from .modules import LLaMAAttention, LLaMABlock, LLaMABlockCollection, LLaMAMLP
from .weights import PackedLinear

# Reference-compatible names (jax_llama/__init__.py:4, model.py:105-772)
FlaxLLaMAForCausalLM = LLaMAForCausalLM
FlaxLLaMAModel = LLaMAModel
FlaxLLaMAAttention = LLaMAAttention
FlaxLLaMAMLP = LLaMAMLP
FlaxLLaMABlock = LLaMABlock
FlaxLLaMABlockCollection = LLaMABlockCollection

__all__ = ["KVCache", "LLaMAForCausalLM", "LLaMAModel", "FlaxLLaMAForCausalLM", "FlaxLLaMAModel",
           "LLaMAAttention", "LLaMAMLP", "LLaMABlock", "LLaMABlockCollection", "FlaxLLaMAAttention",
           "FlaxLLaMAMLP", "FlaxLLaMABlock", "FlaxLLaMABlockCollection",
           "CausalLMOutput", "BaseModelOutput", "PackedLinear", "mask_to_kv_start"]
