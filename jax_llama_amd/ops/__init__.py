"""Op API of the framework.

Every op takes torch tensors and dispatches on the tensor's device:
  * ``cuda`` (ROCm/HIP) tensors -> the hand-written gfx950 HIP kernels in ``_C``
    (``csrc/kernels/*.hip``). If the extension is missing this raises.
  * CPU tensors -> ``ops.reference`` (pure PyTorch; the test/oracle path).

There is exactly one GPU implementation per op (no backend selection, no Triton).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch

from . import autotune
from . import reference as ref
from ._ext import available as ext_available  # noqa: F401
from ._ext import ext

BF16 = torch.bfloat16

# Linear epilogue modes (must match csrc/kernels/common.h)
MODE_STORE = 0
MODE_RESIDUAL = 1
MODE_SWIGLU = 2
MODE_QKV = 3

# GEMV tuning override (0 = built-in heuristic; 1/2/3 = 4/8/16 waves per workgroup)
GEMV_VARIANT = int(os.environ.get("JLA_GEMV_VARIANT", "0"))


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


class _Workspace:
    """Grow-only scratch buffers (per device, per name). Sized during warm-up so that
    nothing is allocated while a decode step is being captured into a hipGraph."""

    def __init__(self):
        self._bufs = {}
        # bumped on every (re)allocation: a captured hipGraph that recorded these buffers' addresses is
        # stale once it changes (runtime/engine.py recaptures)
        self.generation = 0
        self._scope = ""

    @contextlib.contextmanager
    def scope(self, tag: str):
        """Buffers requested inside get their own copies under ``tag``: work issued concurrently on another stream
        (the engine's decode micro-batches) must not share split-K slabs, tickets or attention partials."""
        prev, self._scope = self._scope, tag + "/"
        try:
            yield
        finally:
            self._scope = prev

    def get(self, name: str, numel: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
        key = (self._scope + name, device, dtype)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < numel:
            buf = torch.empty(max(numel, 1), dtype=dtype, device=device)
            self._bufs[key] = buf
            self.generation += 1
        return buf[:numel]

    def get_zeroed(self, name: str, numel: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
        """Zero-initialised on (re)allocation only: for self-resetting device counters."""
        key = ("zeroed:" + self._scope + name, device, dtype)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < numel:
            buf = torch.zeros(max(numel, 1), dtype=dtype, device=device)
            self._bufs[key] = buf
            self.generation += 1
        return buf[:numel]

    def clear(self):
        self._bufs.clear()
        self.generation += 1


workspace = _Workspace()


# ----------------------------------------------------------------------------------
def embedding(ids: torch.Tensor, table: torch.Tensor, mirror: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ids int32 [M] -> fp32 [M, D] rows of the bf16 table (residual stream is fp32).
    ``mirror`` (bf16 [M, D]) also receives the rows: the bf16 copy of the residual stream that
    the next projection reads as its MFMA A operand."""
    if not _is_gpu(table):
        out = ref.embedding(ids, table)
        if mirror is not None:
            mirror.copy_(out.to(BF16))
        return out
    out = torch.empty(ids.numel(), table.shape[1], dtype=torch.float32, device=table.device)
    ext().embedding(ids.reshape(-1).to(torch.int32), table, out, mirror)
    return out


def rms_scale(x: torch.Tensor, eps: float) -> torch.Tensor:
    if not _is_gpu(x):
        return ref.rms_scale(x, eps)
    out = torch.empty(x.shape, dtype=BF16, device=x.device)
    ext().rms_scale(x, out, float(eps))
    return out


def residual_add_(h: torch.Tensor, p: torch.Tensor, mirror: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``h (fp32) += p`` (bf16 or fp32, same shape) and ``mirror = bf16(h)`` in one pass (GPU: one kernel)."""
    if not _is_gpu(h):
        h.add_(p.float().view_as(h))
        if mirror is not None:
            mirror.copy_(h.to(BF16))
        return h
    assert h.is_contiguous() and h.dtype == torch.float32
    if mirror is None or h.numel() % 8:
        h.add_(p.view_as(h))
        if mirror is not None:
            mirror.copy_(h)
        return h
    ext().residual_add(h, p.contiguous(), mirror)
    return h


PREFETCH_GRID = int(os.environ.get("JLA_PREFETCH_GRID", "128"))


def prefetch(t: torch.Tensor) -> None:
    """Load every byte of ``t`` with the default cache policy (warms the Infinity Cache; GPU only, no result)."""
    if _is_gpu(t):
        ext().prefetch(t, PREFETCH_GRID)


def linear_f32(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x [M, K] @ w [N, K]^T`` with fp32 inputs, accumulation and output (precision='highest' lm_head; GPU: the
    exact-f32 MFMA kernel, csrc/kernels/gemm_f32.hip)."""
    if not _is_gpu(x):
        return x.float() @ w.float().t()
    y = torch.empty(x.shape[0], w.shape[0], dtype=torch.float32, device=x.device)
    ext().gemm_f32(x.float().contiguous(), w.float().contiguous(), y)
    return y


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """Stand-alone RMSNorm (fp32 out); the model folds norm weights into GEMMs instead."""
    if not _is_gpu(x):
        return ref.rmsnorm(x, weight, eps)
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    ext().rmsnorm(x.float().contiguous(), weight.float().contiguous(), out, float(eps))
    return out


# ----------------------------------------------------------------------------------
# bounds-checked debug build (JLA_DEBUG_BOUNDS=1 + python build.py --debug-bounds)
BOUNDS_CODES = {0: "token id outside the vocabulary", 1: "KV-cache write past the cache (slot >= T)",
                2: "decode step past the sequence buffer", 3: "attention asked for keys past the cache",
                4: "position outside the RoPE table"}


class BoundsError(RuntimeError):
    pass


def bounds_error(reset: bool = False) -> int:
    """OR of the kernels' out-of-range events since the last reset (bits of BOUNDS_CODES); always 0 unless
    the debug build is loaded. Synchronises the device."""
    if not ext_available():
        return 0
    return int(ext().bounds_error(bool(reset)))


def check_bounds(reset: bool = True):
    """Raise BoundsError naming every out-of-range event the debug build recorded (no-op in release)."""
    if not ext_available() or not getattr(ext(), "DEBUG_BOUNDS", False):
        return
    err = bounds_error(reset)
    if err:
        raise BoundsError("device-side index out of range: " +
                          "; ".join(v for k, v in BOUNDS_CODES.items() if err >> k & 1))


def linear(x: torch.Tensor, w, rms_eps: Optional[float] = None, out_dtype=BF16,
           out: Optional[torch.Tensor] = None, x_packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``y = [inv_rms(x) *] x @ W^T``; ``w`` is a ``models.weights.PackedLinear`` (``x_packed``: optional packed
    copy of x for the packed-x decode variants)."""
    if not _is_gpu(x):
        r = ref.linear(x, w.dense(), rms_eps, out_dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r
    m = x.shape[0]
    if out is None:
        out = torch.empty(m, w.n, dtype=out_dtype, device=x.device)
    _gpu_linear(x, w, out, MODE_STORE, rms_eps, True, None, x_packed)
    return out


def linear_residual(x: torch.Tensor, w, residual: torch.Tensor, rms_eps: Optional[float] = None,
                    accumulate: bool = True, mirror: Optional[torch.Tensor] = None,
                    x_packed: Optional[torch.Tensor] = None, mirror_packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``residual (fp32) += y`` (or ``= y`` when ``accumulate`` is False); ``mirror`` (bf16,
    same shape) receives ``bf16(residual)`` from the same epilogue. Decode (M <= 64): ``x_packed`` is an
    optional packed-layout copy of ``x`` (``packed_rows``) the packed-x GEMV variants may read, and
    ``mirror_packed`` receives a packed copy of the mirror (the next projection's packed x)."""
    if not _is_gpu(x):
        ref.linear_residual(x, w.dense(), residual, rms_eps, accumulate)
        if mirror is not None:
            mirror.copy_(residual.to(BF16))
        return residual
    _gpu_linear(x, w, residual, MODE_RESIDUAL, rms_eps, accumulate, mirror, x_packed, mirror_packed)
    return residual


def linear_swiglu(x: torch.Tensor, w, rms_eps: Optional[float] = None, x_packed: Optional[torch.Tensor] = None,
                  out_packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``silu(x W1^T) * (x W3^T)`` with W1/W3 packed as alternating 16-row tiles (packed-x in/out as in
    ``linear_residual``)."""
    if not _is_gpu(x):
        return ref.linear_swiglu(x, w.dense(), rms_eps)
    out = torch.empty(x.shape[0], w.n // 2, dtype=BF16, device=x.device)
    _gpu_linear(x, w, out, MODE_SWIGLU, rms_eps, True, None, x_packed, out_packed)
    return out


# ---- packed activations (csrc/kernels/common.h pack_off): the MFMA A fragments of a decode activation stored
# contiguously, written beside the row-major copy by the producing GEMV epilogue (or decode attention) and read by
# the packed-x GEMV variants 12-15 -- one 1 KiB load per 16 x 32 fragment instead of 16 half-used 128-B lines
# (profiles/r2_decode_m32_asm_ring.jsonl: o 15.6 -> 10.5 us, down 36.6 -> 30.7 us at M = 32).
PACKED_X = os.environ.get("JLA_PACKED_X", "1") != "0"
PACKED_X_MIN_M = int(os.environ.get("JLA_PACKED_X_MIN_M", "9"))
# up to 64 rows: from 33 rows the tiled split-K GEMM's reduce epilogue writes the packed copies too, so the producers
# keep the tiled GEMM where it wins (w2 at M = 33-64) and the consumers read packed x (profiles/r3_packed_x_m64_ab.jsonl)
PACKED_X_MAX_M = int(os.environ.get("JLA_PACKED_X_MAX_M", "64"))
PACKED_ATT_MAX_M = int(os.environ.get("JLA_PACKED_ATT_MAX_M", "64"))  # attention output only, up to here
SKINNY_M = 64  # decode GEMV rows (csrc: SKINNY_MAX_M): packed copies exist only on that path
XP_VARIANTS = (12, 15, 18, 21, 22, 26)  # packed-x GEMV variants (18 / 26 split-K; 21 / 22: 2x8 / 4x4; 26: 4 tiles x 8
#   waves, K over 4)
SPLIT_VARIANTS = (16, 18, 26)  # split-K GEMV variants (the shared decode workspace holds their slabs)


def packed_rows(m: int) -> int:
    """Rows of a packed activation buffer: the GEMV's m-tiles (1, 2 or 4) x 16."""
    return 16 if m <= 16 else (32 if m <= 32 else 64)


def packed_empty(m: int, cols: int, device) -> torch.Tensor:
    return torch.empty(packed_rows(m), cols, dtype=BF16, device=device)


def _gpu_linear(x, w, out, mode, rms_eps, accumulate, mirror=None, x_packed=None, pack_out=None):
    assert x.is_contiguous() and out.is_contiguous()
    assert x.shape[1] == w.k, (x.shape, w.k)
    m = x.shape[0]
    e = ext()
    if m > e.SKINNY_MAX_M:
        x_packed = pack_out = None
    v = TILED if m > e.SKINNY_MAX_M else _variant(e, x, w, mode, x_packed, pack_out)
    if v == TILED and pack_out is not None and not _tiled_packs(e, m, w.n, w.k, x.device, mode, rms_eps):
        v = 1  # (a plan that cannot pack: the GEMV writes the packed copy)
    if v == TILED:
        _tiled(e, x, w.weight, w.n, w.k, out, mode, rms_eps, accumulate, mirror, pack_out)
    elif x_packed is not None or pack_out is not None:
        ws, tk = _skinny_ws(e, m, w.n, w.k, mode, x.device)
        e.linear_skinny(x, w.weight, w.n, w.k, out, mode, -1.0 if rms_eps is None else float(rms_eps),
                        bool(accumulate), v, ws, tk, mirror, x_packed if v in XP_VARIANTS else None, pack_out)
    else:
        ws, tk = _skinny_ws(e, m, w.n, w.k, mode, x.device)
        e.linear_skinny(x, w.weight, w.n, w.k, out, mode,
                        -1.0 if rms_eps is None else float(rms_eps), bool(accumulate), v, ws, tk, mirror)


def linear_tp_residual(x: torch.Tensor, w, h: torch.Tensor, hb: torch.Tensor, state: int,
                       x_packed: Optional[torch.Tensor] = None, hb_pack: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-parallel decode projection with its all-reduce in the GEMV epilogue (csrc/kernels/gemv.hip
    MODE_TPRESID): ``h (fp32) += sum over the TP group of x @ W^T``, ``hb = bf16(h)`` (+ ``hb_pack``, its packed
    copy). ``state``: a custom all-reduce instance reserved for this path. Bit-identical to ``linear`` (bf16
    partial) + ``TPComm.all_reduce_residual_``, minus one launch and the partial's round trip through HBM."""
    e = ext()
    m = x.shape[0]
    assert x.dtype == BF16 and x.is_contiguous() and m <= e.SKINNY_MAX_M, (x.dtype, x.shape)
    # the exchange lives in the GEMV epilogue: tune among the GEMV variants (``pack_out`` excludes split-K / tiled)
    v = _variant(e, x, w, MODE_RESIDUAL, x_packed, pack_out=True)
    if v == TILED:
        v = 1
    ws = tk = None
    if v in SPLIT_VARIANTS:
        ws, tk = _skinny_ws(e, m, w.n, w.k, MODE_RESIDUAL, x.device)
    e.linear_tp_residual(state, x, w.weight, w.n, w.k, h, hb, v, x_packed if v in XP_VARIANTS else None, hb_pack,
                         ws, tk)
    return h


def tiled_tp_residual(x: torch.Tensor, w, h: torch.Tensor, hb: torch.Tensor, state: int) -> bool:
    """Row-parallel tiled projection with the all-reduce in its split-K reduce (csrc/kernels/gemm.hip
    gemm_reduce_tp_kernel): ``h (fp32) += sum over the TP group of x @ W^T``, ``hb = bf16(h)``. Bit-identical to
    ``linear`` (bf16 partial) + ``TPComm.all_reduce_residual_``. Runs the tuned plan of the unfused partial GEMM; False
    (nothing done) when that plan has no K split (the exchange lives in the reduce)."""
    e = ext()
    m = x.shape[0]
    assert x.dtype == BF16 and x.is_contiguous(), (x.dtype, x.shape)
    ks, tm = autotune.choose_gemm_plan(e, m, w.n, w.k, x.device, MODE_STORE, False)
    if tm not in G5_TILES and ks <= 1:
        return False
    ks, tm, ws = _gemm_ws(e, m, w.n, w.k, x.device, MODE_STORE, False)
    e.gemm_tp_residual(state, x, w.weight, w.n, w.k, h, hb, ks, ws, tm)
    return True


TILED = 7  # decode-kernel "variant" id of the 128x128 MFMA GEMM (split-K for mid M)
# qkv projection without a K split (B = 2048 decode, prefill): RoPE + KV write in the GEMM epilogue (JLA_QKV_DIRECT=0:
# plain GEMM + rope_kv_kernel, for A/B)
QKV_DIRECT = os.environ.get("JLA_QKV_DIRECT", "1") != "0"


def _fused_rms(e, mode, rms_eps) -> bool:
    """The tiled GEMM applies RMSNorm itself (statistics from its own A-fragment reads or a precomputed per-row
    statistic, row scale in the epilogue) except in residual mode."""
    return rms_eps is not None and mode != MODE_RESIDUAL


def _tiled_input(x, rms_eps, fused=False):
    """bf16 A operand of the tiled GEMM: unscaled when the GEMM fuses the norm, else rms-scaled
    (statistics from x's own values) by a separate kernel."""
    if rms_eps is not None and not fused:
        return rms_scale(x, rms_eps)
    return x if x.dtype == BF16 else x.to(BF16)


G5_TILES = (11, 12)  # gemm5 weight-streaming split-K (csrc/kernels/gemm5ws.h): 256- / 128-column workgroups


def _gemm_ws(e, m, n, k, device, mode=MODE_STORE, rms=False):
    """(split-K factor, tile config, workspace) of the tuned plan for this shape and epilogue: the partial slabs of a
    split summed by the reduce kernel (gemm5, tiles 11 / 12: always)."""
    ks, tm = autotune.choose_gemm_plan(e, m, n, k, device, mode, rms)
    if tm in G5_TILES:  # weight-streaming split-K (any split, slabs always): partial slabs + the reduce kernel
        eks = e.gemm5_ksplit(k, ks)
        return ks, tm, workspace.get("gemm_ws", eks * m * (n + 1), torch.float32, device)
    # split-K slabs [ks][m][n] + the fused-RMS partial sums of squares [ks][m]
    ws = workspace.get("gemm_ws", ks * m * (n + 1), torch.float32, device) if ks > 1 else None
    return ks, tm, ws


def _rms_ws(x, fused: bool, ks: int):
    """fp32 [M] scratch for the row statistic of the fused norm, computed ahead of a gemm4 GEMM without a K split
    (csrc/kernels/norm_embed.hip rms_rowinv; the main loop then carries no sum-of-squares work)."""
    if not fused or ks > 1:
        return None
    return workspace.get("gemm_rms", x.shape[0], torch.float32, x.device)


def _tiled(e, x, weight, n, k, out, mode, rms_eps, accumulate, mirror=None, pack_out=None):
    """Tiled MFMA GEMM (prefill, and decode batches > 32): split-K over workgroups when the output has too few
    256x256 tiles to fill the chip (csrc/kernels/gemm.hip). ``pack_out``: the split-K
    reduce epilogue also writes the packed copy of the bf16 output (plans that ``_tiled_packs``)."""
    fused = _fused_rms(e, mode, rms_eps)
    xb = _tiled_input(x, rms_eps, fused)
    ks, tm, ws = _gemm_ws(e, x.shape[0], n, k, x.device, mode, fused)
    e.gemm(xb, weight, n, k, out, mode, bool(accumulate), mirror, ks, ws, float(rms_eps) if fused else -1.0, tm,
           pack_out, _rms_ws(x, fused, ks))


def _tiled_packs(e, m, n, k, device, mode, rms_eps) -> bool:
    """Whether the tiled GEMM's tuned plan for this decode shape can write a packed output copy: the plain split-K
    path, whose reduce kernel runs the epilogue (not ks = 1)."""
    if e is None or m > SKINNY_M or mode not in (MODE_RESIDUAL, MODE_SWIGLU):
        return False
    ks, tm = autotune.choose_gemm_plan(e, m, n, k, device, mode, _fused_rms(e, mode, rms_eps))
    if tm in G5_TILES:
        return True
    return ks > 1


def _variant(e, x, w, mode, x_packed=None, pack_out=None, no_split=False) -> int:
    """Decode-kernel variant for this shape: pinned (JLA_GEMV_VARIANT / ops.GEMV_VARIANT) or
    measured once per shape on the device (ops/autotune.py). With ``x_packed`` the packed-x variants are
    candidates too; with ``pack_out`` only GEMV variants qualify (their epilogue writes the packed copy)."""
    xp_in, p_out = x_packed is not None, pack_out is not None
    if GEMV_VARIANT:
        v = GEMV_VARIANT
        if (v in XP_VARIANTS and not xp_in) or (p_out and v == TILED and not _tiled_packs(
                e, x.shape[0], w.n, w.k, x.device, mode, None if mode == MODE_RESIDUAL else 1e-5)) or (
                v in SPLIT_VARIANTS and (
                no_split or x.dtype != BF16 or w.n // 16 > autotune.SPLIT_MAX_GROUPS)):
            v = 1
        if v == 12 and mode == MODE_SWIGLU:
            v = 15
        return v
    m = x.shape[0]
    pmode = MODE_STORE if mode == MODE_QKV else mode  # QKV epilogue has side effects: tune as STORE
    ws, tk = _skinny_ws(e, m, w.n, w.k, pmode, x.device)
    ncols = w.n // 2 if pmode == MODE_SWIGLU else w.n
    odt = torch.float32 if pmode == MODE_RESIDUAL else BF16
    scratch = workspace.get("tune_out", m * ncols, odt, x.device).view(m, ncols)
    mirror = workspace.get("tune_mirror", m * ncols, BF16, x.device).view(m, ncols) if (
        p_out and pmode == MODE_RESIDUAL) else None
    pscratch = workspace.get("tune_pack", packed_rows(m) * ncols, BF16, x.device).view(-1, ncols) if p_out else None

    tiled_packs = p_out and _tiled_packs(e, m, w.n, w.k, x.device, pmode, None if pmode == MODE_RESIDUAL else 1e-5)

    def run(v, xx, wt):
        if v == TILED:
            _tiled(e, xx, wt, w.n, w.k, scratch, pmode, None if pmode == MODE_RESIDUAL else 1e-5, True, mirror,
                   pscratch if tiled_packs else None)
        elif xp_in or p_out:
            e.linear_skinny(xx, wt, w.n, w.k, scratch, pmode, 1e-5, True, v, ws, tk, mirror,
                            x_packed if v in XP_VARIANTS else None, pscratch)
        else:
            e.linear_skinny(xx, wt, w.n, w.k, scratch, pmode, 1e-5, True, v, ws, tk)

    return autotune.choose(e, x, w, pmode, run, xp_in=xp_in, pack_out=p_out, no_split=no_split,
                           tiled_packs=tiled_packs)


_SK_SIZES = {}


def _skinny_ws(e, m, n, k, mode, device):
    """Split-K partial slabs + self-resetting tickets of the split-K GEMV variants (shared, stream-ordered;
    sized during the eager warm-up step so nothing is allocated under hipGraph capture)."""
    key = (m, n, k, mode)
    sz = _SK_SIZES.get(key)
    if sz is None:
        sz = _SK_SIZES[key] = tuple(e.skinny_workspace(m, n, k, mode))
    floats, tickets = sz
    return (workspace.get("skinny", max(1, floats), torch.float32, device),
            workspace.get_zeroed("skinny_tickets", max(1, tickets), torch.int32, device))


# ----------------------------------------------------------------------------------
def rope_kv_write(qkv: torch.Tensor, table: torch.Tensor, positions: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, slot0, seq_len: int,
                  n_heads: int, n_kv_heads: int, head_dim: int) -> torch.Tensor:
    """Rotate q/k (interleaved RoPE) and write k/v into the cache. ``slot0`` is an int or a
    device int32 tensor of shape [1] (graph-capturable). Returns q ``[B*S, H, Dh]`` bf16."""
    if not _is_gpu(qkv):
        s0 = int(slot0) if not torch.is_tensor(slot0) else int(slot0.item())
        return ref.rope_kv_write(qkv, table, positions, k_cache, v_cache, s0, seq_len,
                                 n_heads, n_kv_heads, head_dim)
    m = qkv.shape[0]
    q = torch.empty(m, n_heads, head_dim, dtype=BF16, device=qkv.device)
    slot_t = _slot_tensor(slot0, qkv.device)
    ext().rope_kv_write(qkv, table, positions.reshape(-1).to(torch.int32), k_cache, v_cache,
                        slot_t, int(seq_len), int(n_heads), int(n_kv_heads), int(head_dim), q)
    return q


def linear_qkv_rope(x: torch.Tensor, w, rms_eps: Optional[float], table: torch.Tensor, positions: torch.Tensor,
                    k_cache: torch.Tensor, v_cache: torch.Tensor, slot0, seq_len: int, n_heads: int,
                    n_kv_heads: int, head_dim: int, x_packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused ``qkv = [inv_rms(x) *] x @ Wqkv^T`` + interleaved RoPE on q/k + KV-cache write at slots
    ``slot0 + s``. Returns rotated q ``[M, H, Dh]`` bf16. Decode (M <= 64) is one kernel (the
    RoPE/cache write is the GEMV epilogue, rotating the fp32 accumulators); prefill runs the MFMA
    GEMM then the RoPE/KV-write kernel."""
    if not _is_gpu(x):
        s0 = int(slot0) if not torch.is_tensor(slot0) else int(slot0.item())
        return ref.linear_qkv_rope(x, w.dense(), rms_eps, table, positions, k_cache, v_cache, s0, seq_len,
                                   n_heads, n_kv_heads, head_dim)
    m = x.shape[0]
    e = ext()
    if m > e.SKINNY_MAX_M:
        x_packed = None
    v = TILED if m > e.SKINNY_MAX_M else _variant(e, x, w, MODE_QKV, x_packed)
    if v == TILED:
        # (same plan key as the plain linear() below: QKV is tuned as a store with the fused norm)
        ks, tm, ws = _gemm_ws(e, m, w.n, w.k, x.device, MODE_STORE, _fused_rms(e, MODE_QKV, rms_eps))
        fused = _fused_rms(e, MODE_QKV, rms_eps)
        if ks == 1 and fused and QKV_DIRECT and e.gemm_qkv_direct_ok(m, tm, w.k):
            # enough tiles, no K split: the GEMM's own RoPE / KV-write epilogue (no qkv round trip, no rope kernel)
            q = torch.empty(m, n_heads, head_dim, dtype=BF16, device=x.device)
            e.gemm_qkv(_tiled_input(x, rms_eps, fused), w.weight, w.n, w.k, table, positions.reshape(-1).to(torch.int32),
                       k_cache, v_cache, _slot_tensor(slot0, x.device), int(seq_len), int(n_heads), int(n_kv_heads),
                       int(head_dim), q, 1, None, float(rms_eps), tm, _rms_ws(x, fused, 1))
            return q
        if ks == 1:  # enough tiles: plain GEMM, then the RoPE/KV-write kernel
            qkv = linear(x, w, rms_eps=rms_eps)
            return rope_kv_write(qkv, table, positions, k_cache, v_cache, slot0, seq_len, n_heads, n_kv_heads,
                                 head_dim)
        q = torch.empty(m, n_heads, head_dim, dtype=BF16, device=x.device)
        e.gemm_qkv(_tiled_input(x, rms_eps, fused), w.weight, w.n, w.k, table, positions.reshape(-1).to(torch.int32),
                   k_cache, v_cache, _slot_tensor(slot0, x.device), int(seq_len), int(n_heads), int(n_kv_heads),
                   int(head_dim), q, ks, ws, float(rms_eps) if fused else -1.0, tm)
        return q
    q = torch.empty(m, n_heads, head_dim, dtype=BF16, device=x.device)
    ws, tk = _skinny_ws(e, m, w.n, w.k, MODE_QKV, x.device)
    e.linear_qkv(x, w.weight, w.n, w.k, -1.0 if rms_eps is None else float(rms_eps), table,
                 positions.reshape(-1).to(torch.int32), k_cache, v_cache, _slot_tensor(slot0, x.device),
                 int(seq_len), int(n_heads), int(n_kv_heads), int(head_dim), q, v, ws, tk,
                 x_packed if v in XP_VARIANTS else None)
    return q


# Fused small-batch decode: the qkv GEMV and the attention in ONE launch (csrc/kernels/gemv.hip qkv_attn_kernel: the
# attention workgroups prefetch their K / V step while the qkv workgroups stream the weights, then wait on the qkv
# workgroups' write-through publish). Used where it measured faster (profiles/r5_qkv_attn_fused_ab.jsonl,
# r5_qkv_attn_fused_split_ab.jsonl): M <= 4 rows with >= 8 query heads per kv head (the 70B tensor-parallel shard: one
# kv head per rank) -- 4.88 -> 4.77 ms per token at B = 1 with the split qkv part; at Llama-3-8B B = 1 (rep 4: 384 qkv
# workgroups) 2.93 -> 3.24 and at the shard's B = 8 / 32 the tuned standalone GEMVs win. JLA_QKV_ATTN=0: never;
# =2: wherever the launch fits.
QKV_ATTN = int(os.environ.get("JLA_QKV_ATTN", "1"))
# K of the fused launch's qkv GEMV over 2 workgroups per column group (the split GEMV's last-arriver sum) when the grid
# still fits the CUs; JLA_QKV_ATTN_SPL=1: one workgroup per column group (3 / 4 splits were built and lost at the 70B
# shard's B = 1: 4.84 / 4.87 vs 4.73 ms per token, profiles/r6_qkv_attn_o_timeline.jsonl, and were removed)
QKV_ATTN_SPL = int(os.environ.get("JLA_QKV_ATTN_SPL", "2"))
# ... and the o projection in the same launch (its workgroups fetch their Wo slice while qkv / attention run, then wait
# for the attention output; the residual or TP-exchange epilogue of the standalone GEMV): M <= 16, 8 query heads per kv
# head, H * Dh <= 1024 -- the 70B tensor-parallel shard. Bit-identical to the two launches, one launch fewer per layer,
# but not faster: the shard's B = 1 step measured 4.76 / 4.79 and 4.73 / 4.76 ms per token without / with it
# (profiles/r6_qkv_attn_o_timeline.jsonl: the o weight stream competes with the qkv GEMV's per-CU stream, and the chain
# after the attention -- go flag, x load, the TP exchange -- is as long as the standalone o GEMV). JLA_QKV_ATTN_O=1: on.
QKV_ATTN_O = int(os.environ.get("JLA_QKV_ATTN_O", "0"))
_CUS = {}


class InLaunchTimeout(RuntimeError):
    """An in-launch wait gave up (the fused qkv + attention launch: a qkv workgroup never published)."""


def check_inlaunch() -> None:
    """Raise InLaunchTimeout if a fused qkv + attention launch recorded a timeout in its error word
    (``qa_sync[2]``, csrc/kernels/gemv.hip qkv_attn_kernel). The device side is sticky -- the counters are no longer
    reset and every later launch writes zeros -- so after a timeout the fused path is refused for the rest of the
    process (the words re-zeroed, the workspace generation bumped so a captured decode graph is re-captured without it).
    Reads device memory (synchronises); called by the engine's host poll."""
    global QKV_ATTN
    for (name, _dev, _dt), buf in list(workspace._bufs.items()):
        if name.startswith("zeroed:") and name.endswith("qa_sync") and buf.is_cuda and int(buf[2].item()):
            QKV_ATTN = 0
            buf.zero_()
            workspace.generation += 1
            raise InLaunchTimeout("fused qkv + attention launch: a wait timed out (the attention workgroups on the qkv "
                                  "workgroups, or the o workgroups on the attention ones; error word qa_sync[2]); the "
                                  "fused path is now off for this process")


def _num_cus(device) -> int:
    key = str(device)
    if key not in _CUS:
        _CUS[key] = torch.cuda.get_device_properties(device).multi_processor_count
    return _CUS[key]


def qkv_attention_o_groups(x: torch.Tensor, w_o, n_heads: int, n_kv_heads: int) -> int:
    """Workgroups of the o projection when the fused decode launch can also run it (``linear_qkv_attention(o=...)``),
    else 0."""
    if not QKV_ATTN_O or not _is_gpu(x):
        return 0
    return int(ext().qkv_attn_o_groups(x.shape[0], n_heads // n_kv_heads, w_o.n, w_o.k))


def qkv_attention_splits(x: torch.Tensor, w, k_cache: torch.Tensor, seq_len: int, n_heads: int, n_kv_heads: int,
                         key_mask: Optional[torch.Tensor] = None, o_groups: int = 0) -> int:
    """Attention workgroups per (row, kv head) pair of the fused qkv + attention launch for this decode step, or 0
    when it does not apply (prefill, a key mask, M > 32, a cache longer than 512, or a grid the CUs cannot hold at
    once). ``o_groups``: the launch also holds the o projection's workgroups (``qkv_attention_o_groups``)."""
    if not QKV_ATTN or seq_len != 1 or key_mask is not None or not _is_gpu(x) or x.dtype != BF16:
        return 0
    m = x.shape[0]
    if QKV_ATTN == 1 and (m > 4 or n_heads < 8 * n_kv_heads):
        return 0
    return int(ext().qkv_attn_splits(m, m, n_kv_heads, n_heads // n_kv_heads, k_cache.shape[2], w.n,
                                     _num_cus(x.device), 1, int(o_groups)))


def _qkv_attention_spl(e, m, w, k_cache, n_heads, n_kv_heads, device, o_groups=0) -> int:
    if QKV_ATTN_SPL > 1 and e.qkv_attn_splits(m, m, n_kv_heads, n_heads // n_kv_heads, k_cache.shape[2], w.n,
                                               _num_cus(device), 2, int(o_groups)) > 0:
        return 2
    return 1


def linear_qkv_attention(x: torch.Tensor, w, rms_eps: Optional[float], table: torch.Tensor, positions: torch.Tensor,
                         k_cache: torch.Tensor, v_cache: torch.Tensor, slot0, kv_start: torch.Tensor, n_heads: int,
                         n_kv_heads: int, head_dim: int, splits: int, x_packed: Optional[torch.Tensor] = None,
                         out_packed: Optional[torch.Tensor] = None, spl: Optional[int] = None,
                         o: Optional[tuple] = None) -> torch.Tensor:
    """One decode token per row: ``linear_qkv_rope`` + ``attention`` in one launch (``qkv_attention_splits`` > 0).
    Returns the attention output ``[B, H * Dh]`` bf16 (``out_packed``: its packed copy for the o projection).
    ``spl``: K of the qkv GEMV over 1 or 2 workgroups per column group (default: 2 where the grid fits).
    ``o = (w_o, h, hb, hb_pack, tp_state)``: the same launch also runs the o projection into the residual
    (``h += out @ Wo^T``, ``hb`` / ``hb_pack`` its bf16 mirrors; ``tp_state`` a fused custom all-reduce instance for the
    tensor-parallel exchange, 0 at world 1) -- ``splits`` must then come from ``qkv_attention_splits(o_groups=...)``."""
    e = ext()
    m = x.shape[0]
    dev = x.device
    rep = n_heads // n_kv_heads
    q = workspace.get("qa_q", m * n_heads * head_dim, BF16, dev).view(m, n_heads, head_dim)
    out = torch.empty(m, n_heads * head_dim, dtype=BF16, device=dev)
    ws = workspace.get("qa_ws", m * n_kv_heads * splits * rep * (head_dim + 4), torch.float32, dev)
    tickets = workspace.get_zeroed("qa_tickets", max(m * n_kv_heads, 64), torch.int32, dev)
    sync = workspace.get_zeroed("qa_sync", int(e.qkv_attn_sync_ints()), torch.int32, dev)
    og = 0 if o is None else int(e.qkv_attn_o_groups(m, rep, o[0].n, o[0].k))
    spl = _qkv_attention_spl(e, m, w, k_cache, n_heads, n_kv_heads, dev, og) if spl is None else int(spl)
    sk_ws = sk_tk = None
    if spl > 1:
        sk_ws, sk_tk = _skinny_ws(e, m, w.n, w.k, MODE_QKV, dev)
    ow = oh = ohb = ohp = None
    on = ok = 0
    tp_state = 0
    if o is not None:
        wo, oh, ohb, ohp, tp_state = o
        ow, on, ok = wo.weight, wo.n, wo.k
    e.linear_qkv_attn(x, w.weight, w.n, w.k, -1.0 if rms_eps is None else float(rms_eps), table,
                      positions.reshape(-1).to(torch.int32), k_cache, v_cache, _slot_tensor(slot0, dev), n_heads,
                      n_kv_heads, head_dim, q, kv_start, out, out_packed, ws, tickets, sync, k_cache.shape[2], splits,
                      x_packed, spl, sk_ws, sk_tk, ow, on, ok, oh, ohb, ohp, int(tp_state or 0))
    return out


def attention_packs(q: torch.Tensor, k_cache: torch.Tensor, key_mask: Optional[torch.Tensor] = None) -> bool:
    """Whether ``attention(..., out_packed=...)`` can write the packed copy for this decode shape (with a key mask
    only the small-batch kernels, v3 / v5, do: mid-batch rows then go to v2)."""
    bsz, s, h, _ = q.shape
    if s != 1:
        return False
    e = ext()
    if key_mask is not None and bsz > 32:
        return False
    return bool(e.attn_decode_packs(bsz, k_cache.shape[1], h // k_cache.shape[1]))


def attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, slot0, kv_start: torch.Tensor,
              key_mask: Optional[torch.Tensor] = None, max_kv: Optional[int] = None,
              out_packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Causal/padded attention of ``q [B, S, H, Dh]`` (queries at cache slots slot0+s)
    against ``[B, Hkv, T, Dh]`` caches. Returns ``[B*S, H*Dh]`` bf16.

    ``max_kv`` bounds the number of key slots the launch must cover (defaults to the cache
    length T so the launch shape is static and graph-capturable)."""
    bsz, s, h, dh = q.shape
    if not _is_gpu(q):
        s0 = int(slot0) if not torch.is_tensor(slot0) else int(slot0.item())
        return ref.attention(q, k_cache, v_cache, s0, kv_start, key_mask).reshape(bsz * s, h * dh)
    out = torch.empty(bsz * s, h * dh, dtype=BF16, device=q.device)
    slot_t = _slot_tensor(slot0, q.device)
    t_cap = int(max_kv) if max_kv is not None else k_cache.shape[2]
    e = ext()
    if s == 1:
        hkv = k_cache.shape[1]
        nsplit = e.attn_decode_splits(bsz, hkv, t_cap, h // hkv)
        ws = workspace.get("attn_decode", bsz * h * nsplit * (dh + 4), torch.float32, q.device)
        tickets = workspace.get_zeroed("attn_tickets", bsz * hkv, torch.int32, q.device)
        e.attn_decode(q, k_cache, v_cache, slot_t, kv_start, key_mask, out, ws, tickets, t_cap, nsplit, out_packed)
    else:
        e.attn_prefill(q, k_cache, v_cache, slot_t, kv_start, key_mask, out)
    return out


_SLOT_CACHE = {}


def _slot_tensor(slot0, device):
    if torch.is_tensor(slot0):
        return slot0
    # Host int -> small device tensor (not graph-capturable; the engine passes tensors).
    t = torch.tensor([int(slot0)], dtype=torch.int32, device=device)
    return t


# ----------------------------------------------------------------------------------
def argmax(logits: torch.Tensor):
    """Row argmax (first max index, like ``jnp.argmax``). Returns (idx int32[B], val fp32[B])."""
    if not _is_gpu(logits):
        v, i = logits.float().max(-1)
        return ref.argmax(logits), v
    b = logits.shape[0]
    idx = torch.empty(b, dtype=torch.int32, device=logits.device)
    val = torch.empty(b, dtype=torch.float32, device=logits.device)
    ext().argmax(logits, idx, val)
    return idx, val


ARGMAX_FUSED_MIN_M = 256  # one 256-row tile or more: the tiled GEMM is the lm_head kernel anyway
# decode M <= 64: the argmax runs in the lm_head GEMV's epilogue (per-16-column partials); JLA_SKINNY_ARGMAX=0 off
SKINNY_ARGMAX = os.environ.get("JLA_SKINNY_ARGMAX", "1") != "0"


def linear_argmax(x: torch.Tensor, w, rms_eps: Optional[float] = None):
    """Greedy token of ``[inv_rms(x) *] x @ W^T`` (the lm_head): ``(idx int32[M], val fp32[M])``, first
    max like ``jnp.argmax``. On the GPU the argmax runs in the GEMM epilogue and the fp32 logits never
    reach HBM: in the decode GEMV's (M <= 64, ``linear_skinny_argmax``) or in the tiled GEMM's (from
    ARGMAX_FUSED_MIN_M rows, ``gemm_argmax``); in between ``linear`` + ``argmax``."""
    m = x.shape[0]
    if not _is_gpu(x):
        return argmax(linear(x, w, rms_eps, out_dtype=torch.float32))
    if m <= ext().SKINNY_MAX_M and SKINNY_ARGMAX:
        e = ext()
        v = _variant(e, x, w, MODE_STORE, no_split=True)  # the logits GEMV's main loop: its tuned variant applies
        if v in (1, 2, 3, 5, 6, 8, 9, 20):
            part = workspace.get("skinny_argmax", m * (w.n // 16) * 2, torch.float32, x.device)
            idx = torch.empty(m, dtype=torch.int32, device=x.device)
            val = torch.empty(m, dtype=torch.float32, device=x.device)
            e.linear_skinny_argmax(x, w.weight, w.n, w.k, -1.0 if rms_eps is None else float(rms_eps), v, part, idx,
                                   val)
            return idx, val
    if m < ARGMAX_FUSED_MIN_M:
        return argmax(linear(x, w, rms_eps, out_dtype=torch.float32))
    e = ext()
    assert x.is_contiguous() and x.shape[1] == w.k, (x.shape, w.k)
    xb = x if x.dtype == BF16 else x.to(BF16)
    ws = workspace.get("gemm_argmax", e.gemm_argmax_workspace(m, w.n), torch.float32, x.device)
    idx = torch.empty(m, dtype=torch.int32, device=x.device)
    val = torch.empty(m, dtype=torch.float32, device=x.device)
    e.gemm_argmax(xb, w.weight, w.n, w.k, ws, -1.0 if rms_eps is None else float(rms_eps), idx, val,
                  _rms_ws(x, rms_eps is not None, 1))
    return idx, val


SAMPLER_MAX_K = 64


def topk_candidates(logits: torch.Tensor, k: int, idx_offset: int = 0):
    """Sorted top-``k`` (values fp32 [B, k], global indices int32 [B, k]) of fp32 logits on the
    device: per-8192-chunk prefiltered radix select + one merge (csrc/kernels/topk_sample.hip)."""
    if not _is_gpu(logits):
        v, i = ref.topk_sorted(logits, k)
        return v, i + idx_offset
    e = ext()
    b, v = logits.shape
    c = e.topk_chunks(v) * k
    cv = workspace.get("topk_cv", b * c, torch.float32, logits.device).view(b, c)
    ci = workspace.get("topk_ci", b * c, torch.int32, logits.device).view(b, c)
    e.topk_chunk(logits, k, int(idx_offset), cv, ci)
    out_v = torch.empty(b, k, dtype=torch.float32, device=logits.device)
    out_i = torch.empty(b, k, dtype=torch.int32, device=logits.device)
    e.topk_merge(cv, ci, k, 0, out_v=out_v, out_i=out_i)
    return out_v, out_i


def topk_sample(logits: torch.Tensor, k: int, temperature: float, top_p: float, seed: int,
                step: torch.Tensor, comm=None) -> torch.Tensor:
    """temperature -> top-k -> top-p -> categorical on the device, exact under vocab-parallel TP
    (each rank's top-k is all-gathered, 2*k*4 bytes per row, and merged again; every rank draws
    the same token from the same Philox stream). ``step`` is a device int32[1] (the decode
    loop's cur_len) so the call is hipGraph-capturable. Returns int32 [B]."""
    b, v = logits.shape
    tp = comm.size if comm is not None else 1
    if not _is_gpu(logits):
        if tp > 1:
            full = comm.all_gather(logits.float().contiguous()).permute(1, 0, 2).reshape(b, -1)
        else:
            full = logits
        return ref.topk_sample(full, k, temperature, 1.0 if top_p is None else top_p, seed, int(step.reshape(-1)[0]))
    e = ext()
    kl = min(k, v)  # per-rank candidates (tp * kl >= k)
    c = e.topk_chunks(v) * kl
    cv = workspace.get("topk_cv", b * c, torch.float32, logits.device).view(b, c)
    ci = workspace.get("topk_ci", b * c, torch.int32, logits.device).view(b, c)
    e.topk_chunk(logits, kl, int(comm.rank * v) if tp > 1 else 0, cv, ci)
    if tp > 1:
        lv = torch.empty(b, kl, dtype=torch.float32, device=logits.device)
        li = torch.empty(b, kl, dtype=torch.int32, device=logits.device)
        e.topk_merge(cv, ci, kl, 0, out_v=lv, out_i=li)
        cv, ci = comm.gather_topk(lv, li)  # custom gather kernel (graph-capturable) on the GPU
    nxt = torch.empty(b, dtype=torch.int32, device=logits.device)
    e.topk_merge(cv, ci, k, 1, nxt=nxt, temperature=float(temperature),
                 top_p=1.0 if top_p is None else float(top_p), seed=int(seed) & ((1 << 63) - 1), step=step)
    return nxt
