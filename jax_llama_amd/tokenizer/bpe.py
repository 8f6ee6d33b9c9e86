"""tiktoken-compatible byte-pair encoding.

tiktoken (a Rust extension) is not available in this environment, so the merge core is our
own C++ (``csrc/bpe/bpe.cpp`` -> ``jax_llama_amd/_bpe*.so``, built by ``build.py``). The
regex pre-tokeniser runs on the ``regex`` module (it supports ``\\p{L}``/``\\p{N}``).
``PyBPE`` is a pure-Python implementation of the same algorithm used as the test oracle.

Algorithm (tiktoken ``byte_pair_encode``): a piece found whole in the rank table is one
token; otherwise start from single bytes and repeatedly merge the adjacent pair whose
concatenation has the lowest rank until no adjacent pair is in the table.
"""
from __future__ import annotations

import base64
import importlib
import logging
from typing import AbstractSet, Collection, Dict, Iterable, List, Optional, Union

import regex

logger = logging.getLogger(__name__)


def load_tiktoken_bpe(path: str) -> Dict[bytes, int]:
    """Parse a tiktoken rank file: one ``base64(token) rank`` pair per line."""
    ranks: Dict[bytes, int] = {}
    with open(path, "rb") as f:
        for line in f.read().splitlines():
            if not line:
                continue
            tok, rank = line.split()
            ranks[base64.b64decode(tok)] = int(rank)
    return ranks


def save_tiktoken_bpe(ranks: Dict[bytes, int], path: str) -> None:
    with open(path, "wb") as f:
        for tok, rank in sorted(ranks.items(), key=lambda kv: kv[1]):
            f.write(base64.b64encode(tok) + b" " + str(rank).encode() + b"\n")


class PyBPE:
    """Pure-Python reference merge core (oracle for the C++ one)."""

    def __init__(self, ranks: Dict[bytes, int]):
        self.ranks = ranks

    def encode_piece(self, piece: bytes) -> List[int]:
        r = self.ranks.get(piece)
        if r is not None:
            return [r]
        parts = [bytes([b]) for b in piece]
        while len(parts) > 1:
            best, best_i = None, -1
            for i in range(len(parts) - 1):
                rr = self.ranks.get(parts[i] + parts[i + 1])
                if rr is not None and (best is None or rr < best):
                    best, best_i = rr, i
            if best is None:
                break
            parts[best_i:best_i + 2] = [parts[best_i] + parts[best_i + 1]]
        return [self.ranks[p] for p in parts]

    def encode_pieces(self, pieces: Iterable[bytes]) -> List[int]:
        out: List[int] = []
        for p in pieces:
            out.extend(self.encode_piece(p))
        return out


def _native_core(ranks: Dict[bytes, int]):
    try:
        mod = importlib.import_module("jax_llama_amd._bpe")
    except ImportError as e:
        logger.warning("native BPE core not built (%s); using the Python merge loop", e)
        return None
    core = mod.BPE()
    core.load(list(ranks.keys()), list(ranks.values()))
    return core


class Encoding:
    """Minimal ``tiktoken.Encoding`` equivalent: ``encode``, ``decode``, ``n_vocab``."""

    def __init__(self, name: str, pat_str: str, mergeable_ranks: Dict[bytes, int],
                 special_tokens: Dict[str, int], native: bool = True):
        self.name = name
        self._pat = regex.compile(pat_str)
        self._ranks = mergeable_ranks
        self._special = dict(special_tokens)
        self._decoder: Dict[int, bytes] = {v: k for k, v in mergeable_ranks.items()}
        for s, i in special_tokens.items():
            self._decoder[i] = s.encode("utf-8")
        self._core = _native_core(mergeable_ranks) if native else None
        self._py = PyBPE(mergeable_ranks)
        self._special_re = (regex.compile("|".join(regex.escape(s) for s in
                                                    sorted(special_tokens, key=len, reverse=True)))
                            if special_tokens else None)
        self.n_vocab = max(max(mergeable_ranks.values(), default=-1),
                           max(special_tokens.values(), default=-1)) + 1

    @property
    def native(self) -> bool:
        return self._core is not None

    @property
    def mergeable_ranks(self) -> Dict[bytes, int]:
        return self._ranks

    @property
    def special_tokens_set(self) -> AbstractSet[str]:
        return set(self._special)

    def _encode_ordinary(self, text: str) -> List[int]:
        pieces = [m.encode("utf-8") for m in self._pat.findall(text)]
        if self._core is not None:
            return self._core.encode_pieces(pieces)
        return self._py.encode_pieces(pieces)

    def encode_ordinary(self, text: str) -> List[int]:
        return self._encode_ordinary(text)

    def encode(self, text: str, *, allowed_special: Union[str, AbstractSet[str]] = frozenset(),
               disallowed_special: Union[str, Collection[str]] = "all") -> List[int]:
        if allowed_special == "all":
            allowed_special = set(self._special)
        if disallowed_special == "all":
            disallowed_special = set(self._special) - set(allowed_special)
        if disallowed_special:
            for s in disallowed_special:
                if s in text:
                    raise ValueError(f"Encountered text corresponding to disallowed special token {s!r}")
        if not allowed_special or self._special_re is None:
            return self._encode_ordinary(text)
        out: List[int] = []
        start = 0
        for m in self._special_re.finditer(text):
            if m.group(0) not in allowed_special:
                continue
            out.extend(self._encode_ordinary(text[start:m.start()]))
            out.append(self._special[m.group(0)])
            start = m.end()
        out.extend(self._encode_ordinary(text[start:]))
        return out

    def decode_bytes(self, tokens: Iterable[int]) -> bytes:
        return b"".join(self._decoder[int(t)] for t in tokens)

    def decode(self, tokens: Iterable[int], errors: str = "replace") -> str:
        return self.decode_bytes(tokens).decode("utf-8", errors=errors)
