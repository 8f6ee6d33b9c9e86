"""Loader for the in-tree native HIP extension (``jax_llama_amd/_C*.so``).

The extension is built by ``python build.py`` (hipcc, ``--offload-arch=gfx950``). Every op
that receives a GPU tensor goes through it; if it is missing on a GPU we raise instead of
silently running a slower path (the CPU reference path is only used for CPU tensors).
``JLA_DEBUG_BOUNDS=1`` loads the bounds-checked debug build ``_C_dbg`` instead
(``python build.py --debug-bounds``; see ``ops.check_bounds``).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

_EXT = None
_ERR: Optional[BaseException] = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return
    try:
        import torch  # noqa: F401  (libtorch / libamdhip64 must be loaded first)
        name = "_C_dbg" if os.environ.get("JLA_DEBUG_BOUNDS", "0") == "1" else "_C"
        _EXT = importlib.import_module("jax_llama_amd." + name)
        # A/B knobs for tools: JLA_ATTN_IMPL=<impl>[:<waves_target>] (csrc/kernels/attn_decode.hip attn_set_impl)
        if os.environ.get("JLA_ATTN_IMPL"):
            impl, _, tgt = os.environ["JLA_ATTN_IMPL"].partition(":")
            _EXT.attn_set_impl(int(impl), int(tgt or 0))
    except BaseException as e:  # ImportError, OSError (undefined symbol), ...
        _ERR = e


def ext():
    """Return the native module or raise a loud error explaining how to build it."""
    _load()
    if _EXT is None:
        raise RuntimeError(
            "jax_llama_amd native HIP extension is not available "
            f"({type(_ERR).__name__}: {_ERR}). Build it with `python build.py` "
            "(requires hipcc, targets gfx950). GPU tensors are never run on a fallback path."
        )
    return _EXT


def available() -> bool:
    _load()
    return _EXT is not None


def so_path() -> Optional[str]:
    _load()
    return getattr(_EXT, "__file__", None) if _EXT is not None else None


def reset_for_tests():  # pragma: no cover - debugging helper
    global _EXT, _ERR
    _EXT, _ERR = None, None
    os.environ.pop("JLA_FORCE_NO_EXT", None)
