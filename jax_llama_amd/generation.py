"""``LLaMA`` text generator — same API and post-processing as the reference
(``/root/reference/jax_llama/generation.py:15-79``):

  * ``generate(tokens, attention_mask, max_gen_len, temperature=0.8, top_p=0.95)`` builds a
    generation config with ``do_sample = temperature != 0``, ``max_length = S + max_gen_len``,
    ``pad = eos = tokenizer.eos_id`` and the HF default top-k of 50 (``:28-41``);
  * ``generate_from_str(prompts, ...)`` encodes with BOS, **left-pads with eos_id**, uses
    ``mask = tokens != eos_id`` and decodes each row from its first BOS, cut to
    ``len(prompt) + max_gen_len`` and at the first EOS — the prompt is included (``:47-79``).

Differences by design: no debug prints; the decode loop runs on the hipGraph engine; with
tensor parallelism every rank calls these methods (SPMD) and rank-0's tokenizer output is
what is returned everywhere (token ids are identical on all ranks by construction).
"""
from __future__ import annotations

from typing import Any, List, Optional, Union

import torch

from .parallel.partition import P, Mesh, gather_dp, with_named_sharding_constraint
from .runtime.engine import GenerationConfig


class LLaMA:
    def __init__(self, params: Optional[Any], model, tokenizer, mesh: Optional[Mesh] = None):
        self.params = params
        self.model = model
        self.tokenizer = tokenizer
        self.mesh = mesh

    def generate(self, tokens, attention_mask, max_gen_len: int, temperature: float = 0.8,
                 top_p: float = 0.95, seed: int = 0) -> torch.Tensor:
        tokens = torch.as_tensor(tokens, dtype=torch.int32) if not torch.is_tensor(tokens) else tokens
        attention_mask = (torch.as_tensor(attention_mask, dtype=torch.int32)
                          if not torch.is_tensor(attention_mask) else attention_mask)
        tokens = with_named_sharding_constraint(tokens, self.mesh, P("dp", None))
        attention_mask = with_named_sharding_constraint(attention_mask, self.mesh, P("dp", None))
        gc = GenerationConfig(
            num_beams=1,
            do_sample=temperature != 0.0,
            max_length=max_gen_len + tokens.shape[1],
            pad_token_id=self.tokenizer.eos_id,
            eos_token_id=self.tokenizer.eos_id,
            temperature=temperature,
            top_p=top_p,
            seed=seed,
        )
        out = self.model.generate(tokens, attention_mask=attention_mask, generation_config=gc)
        # the reference's output constraint P("dp", None) keeps the batch split across dp replicas;
        # here every replica gets the whole batch back (all-gather over the dp group when there is one)
        return gather_dp(out.sequences, self.mesh)

    def generate_from_str(self, prompts: List[str], max_gen_len: int, temperature: float = 0.8,
                          top_p: float = 0.95, seed: int = 0) -> List[str]:
        tok = self.tokenizer
        prompt_tokens = [tok.encode(x, bos=True, eos=False) for x in prompts]
        max_prompt = max(len(t) for t in prompt_tokens)
        tokens = torch.full((len(prompts), max_prompt), tok.eos_id, dtype=torch.int32)
        for i, t in enumerate(prompt_tokens):
            tokens[i, max_prompt - len(t):] = torch.tensor(t, dtype=torch.int32)  # left pad
        attention_mask = (tokens != tok.eos_id).to(torch.int32)
        out_tokens = self.generate(tokens, attention_mask, max_gen_len, temperature, top_p, seed)
        # rows of this dp replica only when the outputs could not be gathered (no process group)
        row0 = 0 if out_tokens.shape[0] == len(prompts) else self.mesh.dp_rank * out_tokens.shape[0]
        decoded = []
        for i, t in enumerate(out_tokens.tolist()):
            t = t[t.index(tok.bos_id):]
            t = t[: len(prompt_tokens[row0 + i]) + max_gen_len]
            try:
                t = t[: t.index(tok.eos_id)]
            except ValueError:
                pass
            decoded.append(tok.decode(t))
        return decoded
