"""LLaMA-1/2 SentencePiece tokenizer (reference ``jax_llama/llama2_tokenizer.py:14-71``):
same constructor, ``encode(s, bos, eos)``, ``decode``, ``__len__`` and the
``bos_id/eos_id/pad_id/n_words`` attributes. SentencePiece's own C++ core does the work."""
from __future__ import annotations

import logging
import os
from typing import List

logger = logging.getLogger(__name__)


class Tokenizer:
    def __init__(self, model_path: str):
        from sentencepiece import SentencePieceProcessor

        assert os.path.isfile(model_path), model_path
        self.sp_model = SentencePieceProcessor(model_file=model_path)
        logger.info(f"Reloaded SentencePiece model from {model_path}")
        self.n_words: int = self.sp_model.vocab_size()
        self.bos_id: int = self.sp_model.bos_id()
        self.eos_id: int = self.sp_model.eos_id()
        self.pad_id: int = self.sp_model.pad_id()
        logger.info(f"#words: {self.n_words} - BOS ID: {self.bos_id} - EOS ID: {self.eos_id}")
        assert self.sp_model.vocab_size() == self.sp_model.get_piece_size()

    def encode(self, s: str, bos: bool, eos: bool) -> List[int]:
        assert type(s) is str
        t = self.sp_model.encode(s)
        if bos:
            t = [self.bos_id] + t
        if eos:
            t = t + [self.eos_id]
        return t

    def decode(self, t: List[int]) -> str:
        return self.sp_model.decode(t)

    def __len__(self) -> int:
        return self.sp_model.vocab_size()
