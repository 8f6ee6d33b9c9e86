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
from typing import AbstractSet, Collection, Dict, List, Literal, Sequence, TypedDict, Union

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

    # guards against pathological inputs (reference llama3_tokenizer.py:131-146): the text is encoded in
    # windows of at most WINDOW_CHARS code points, and a run of more than MAX_RUN_CHARS characters of one
    # class (whitespace / non-whitespace) is cut into MAX_RUN_CHARS-sized pieces
    WINDOW_CHARS = 400_000
    MAX_RUN_CHARS = 25_000

    def encode(self, s: str, *, bos: bool, eos: bool,
               allowed_special: Union[Literal["all"], AbstractSet[str]] = set(),
               disallowed_special: Union[Literal["all"], Collection[str]] = ()) -> List[int]:
        if not isinstance(s, str):
            raise TypeError(f"expected str, got {type(s).__name__}")
        bounds = chunk_bounds(s, self.WINDOW_CHARS, self.MAX_RUN_CHARS)
        ids: List[int] = [self.bos_id] if bos else []
        for lo, hi in zip(bounds, bounds[1:]):
            ids += self.model.encode(s[lo:hi], allowed_special=allowed_special,
                                     disallowed_special=disallowed_special)
        if eos:
            ids.append(self.eos_id)
        return ids

    def decode(self, t: Sequence[int]) -> str:
        return self.model.decode(list(t))

    def __len__(self) -> int:
        return self.n_words


def _chunk_bounds_py(text: str, window: int, max_run: int) -> List[int]:
    """Python twin of the C++ ``chunk_bounds`` (used when the native core is not built)."""
    cuts = [0]
    for w0 in range(0, len(text), window):
        w1 = min(len(text), w0 + window)
        if w0:
            cuts.append(w0)
        a = w0
        while a < w1:
            sp = text[a].isspace()
            b = a + 1
            while b < w1 and text[b].isspace() == sp:
                b += 1
            cuts.extend(range(a + max_run, b, max_run))
            a = b
    if text:
        cuts.append(len(text))
    return cuts


def chunk_bounds(text: str, window: int, max_run: int) -> List[int]:
    try:
        from .._bpe import chunk_bounds as native
    except ImportError:
        return _chunk_bounds_py(text, window, max_run)
    return native(text, window, max_run)


class ChatFormat:
    """Llama-3 chat template (reference ``llama3_tokenizer.py:205-232``): every message is
    ``<|start_header_id|> role <|end_header_id|> "\n\n" content.strip() <|eot_id|>``; a dialog prompt is
    ``<|begin_of_text|>`` + its messages + an open assistant header."""

    def __init__(self, tokenizer: Tokenizer):
        self.tokenizer = tokenizer

    def _special(self, name: str) -> int:
        return self.tokenizer.special_tokens[f"<|{name}|>"]

    def _text(self, text: str) -> List[int]:
        return self.tokenizer.encode(text, bos=False, eos=False)

    def encode_header(self, message: Message) -> List[int]:
        return [self._special("start_header_id"), *self._text(message["role"]), self._special("end_header_id"),
                *self._text("\n\n")]

    def encode_message(self, message: Message) -> List[int]:
        return self.encode_header(message) + self._text(message["content"].strip()) + [self._special("eot_id")]

    def encode_dialog_prompt(self, dialog: Dialog) -> List[int]:
        body = [tok for m in dialog for tok in self.encode_message(m)]
        return [self._special("begin_of_text"), *body, *self.encode_header({"role": "assistant", "content": ""})]
