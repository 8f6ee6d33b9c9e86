"""Llama-3 tokenizer and chat format (reference ``jax_llama/llama3_tokenizer.py:38-232``).

Same public surface: ``Tokenizer(model_path)`` over a tiktoken-format rank file with the 256
special tokens appended after the base ranks, ``encode(s, *, bos, eos, allowed_special,
disallowed_special)`` with the 400k-char / 25k-same-class chunking, ``decode``, ``__len__``,
``bos_id/eos_id/pad_id(-1)/n_words/stop_tokens/special_tokens``; ``ChatFormat`` with
``encode_header/encode_message/encode_dialog_prompt``. The BPE merge core is our C++
(``tokenizer/bpe.py``) instead of tiktoken's Rust.
"""
from __future__ import annotations

import logging
import os
from pathlib import Path
from typing import AbstractSet, Collection, Dict, Iterator, List, Literal, Sequence, TypedDict, Union

from .bpe import Encoding, load_tiktoken_bpe

logger = logging.getLogger(__name__)

Role = Literal["system", "user", "assistant"]


class Message(TypedDict):
    role: Role
    content: str


Dialog = Sequence[Message]


class Tokenizer:
    special_tokens: Dict[str, int]
    num_reserved_special_tokens = 256
    pat_str = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
               r"|\s*[\r\n]+|\s+(?!\S)|\s+")

    def __init__(self, model_path: str, native: bool = True):
        assert os.path.isfile(model_path), model_path
        mergeable_ranks = load_tiktoken_bpe(model_path)
        num_base_tokens = len(mergeable_ranks)
        special_tokens = [
            "<|begin_of_text|>",
            "<|end_of_text|>",
            "<|reserved_special_token_0|>",
            "<|reserved_special_token_1|>",
            "<|reserved_special_token_2|>",
            "<|reserved_special_token_3|>",
            "<|start_header_id|>",
            "<|end_header_id|>",
            "<|reserved_special_token_4|>",
            "<|eot_id|>",
        ] + [f"<|reserved_special_token_{i}|>" for i in range(5, self.num_reserved_special_tokens - 5)]
        self.special_tokens = {tok: num_base_tokens + i for i, tok in enumerate(special_tokens)}
        self.model = Encoding(name=Path(model_path).name, pat_str=self.pat_str,
                              mergeable_ranks=mergeable_ranks, special_tokens=self.special_tokens,
                              native=native)
        logger.info(f"Reloaded tiktoken-format model from {model_path}")
        self.n_words: int = self.model.n_vocab
        self.bos_id: int = self.special_tokens["<|begin_of_text|>"]
        self.eos_id: int = self.special_tokens["<|end_of_text|>"]
        self.pad_id: int = -1
        self.stop_tokens = {self.special_tokens["<|end_of_text|>"], self.special_tokens["<|eot_id|>"]}

    def encode(self, s: str, *, bos: bool, eos: bool,
               allowed_special: Union[Literal["all"], AbstractSet[str]] = set(),
               disallowed_special: Union[Literal["all"], Collection[str]] = ()) -> List[int]:
        assert type(s) is str
        TIKTOKEN_MAX_ENCODE_CHARS = 400_000
        MAX_NO_WHITESPACES_CHARS = 25_000
        substrs = (
            substr
            for i in range(0, len(s), TIKTOKEN_MAX_ENCODE_CHARS)
            for substr in self._split_whitespaces_or_nonwhitespaces(
                s[i: i + TIKTOKEN_MAX_ENCODE_CHARS], MAX_NO_WHITESPACES_CHARS)
        )
        t: List[int] = []
        for substr in substrs:
            t.extend(self.model.encode(substr, allowed_special=allowed_special,
                                       disallowed_special=disallowed_special))
        if bos:
            t.insert(0, self.bos_id)
        if eos:
            t.append(self.eos_id)
        return t

    def decode(self, t: Sequence[int]) -> str:
        return self.model.decode(list(t))

    def __len__(self) -> int:
        return self.n_words

    @staticmethod
    def _split_whitespaces_or_nonwhitespaces(s: str, max_consecutive_slice_len: int) -> Iterator[str]:
        current_slice_len = 0
        current_slice_is_space = s[0].isspace() if len(s) > 0 else False
        slice_start = 0
        for i in range(len(s)):
            is_now_space = s[i].isspace()
            if current_slice_is_space ^ is_now_space:
                current_slice_len = 1
                current_slice_is_space = is_now_space
            else:
                current_slice_len += 1
                if current_slice_len > max_consecutive_slice_len:
                    yield s[slice_start:i]
                    slice_start = i
                    current_slice_len = 1
        yield s[slice_start:]


class ChatFormat:
    def __init__(self, tokenizer: Tokenizer):
        self.tokenizer = tokenizer

    def encode_header(self, message: Message) -> List[int]:
        tokens = [self.tokenizer.special_tokens["<|start_header_id|>"]]
        tokens.extend(self.tokenizer.encode(message["role"], bos=False, eos=False))
        tokens.append(self.tokenizer.special_tokens["<|end_header_id|>"])
        tokens.extend(self.tokenizer.encode("\n\n", bos=False, eos=False))
        return tokens

    def encode_message(self, message: Message) -> List[int]:
        tokens = self.encode_header(message)
        tokens.extend(self.tokenizer.encode(message["content"].strip(), bos=False, eos=False))
        tokens.append(self.tokenizer.special_tokens["<|eot_id|>"])
        return tokens

    def encode_dialog_prompt(self, dialog: Dialog) -> List[int]:
        tokens = [self.tokenizer.special_tokens["<|begin_of_text|>"]]
        for message in dialog:
            tokens.extend(self.encode_message(message))
        tokens.extend(self.encode_header({"role": "assistant", "content": ""}))
        return tokens
