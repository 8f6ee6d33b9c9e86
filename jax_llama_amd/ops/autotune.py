"""Per-shape selection among the decode linear kernels, measured on the device at first use.

The decode GEMV (``csrc/kernels/gemv.hip``: K split across the waves of a workgroup, 1/2/4 tiles per workgroup, optional
K split across workgroups, row-major or packed activations) and the tiled MFMA GEMM compete; which one streams the
weights fastest depends on (M, N, K) in ways that are cheaper to measure than to model (rocprof studies:
profiles/README.md). Variants never picked at a bench or latency shape were removed in round 4
(profiles/r4_variant_pruning.md). The first eager call of a shape times every
candidate on a rotating set of scratch weights (> Infinity Cache, so each call streams from HBM,
as in a real decode step) and caches the winner. Never runs under hipGraph capture; shapes first
seen during capture fall back to the static heuristic.

Variants: 1 = GEMV 4 waves (1 or 2 tiles/WG), 5 = GEMV 4 tiles/WG, 6 = GEMV 2 tiles/WG, 10 = 2 tiles with a doubled
register ring (M > 16, bf16 activations), 20 = 2 tiles x 8 waves, 16 = K over 2 workgroups, packed-x 12 / 15 / 18 / 21 /
22 / 26, 7 = tiled MFMA GEMM with split-K (gemm.hip; a candidate for M > 16, always used for M > 64). ``JLA_GEMV_VARIANT`` pins one; ``JLA_AUTOTUNE=0`` disables tuning.

Shipped picks: ``ops/tune_gfx950.json`` (measured on an MI355X for the bench, latency and tensor-parallel shapes) is
loaded first, so plans are identical on every box and nothing is measured for those shapes; shapes it lacks are
measured as above.

Tensor parallelism: inside ``tp_scope(comm)`` (the model's forward under TP) a decision is collective -- rank 0
of the TP group measures and broadcasts its choice, so every rank runs the same plans (a rank on a slower plan
would set the pace of every collective). Persistence: decisions are kept per (arch, shape) in a JSON table
(``JLA_TUNE_FILE``, default ``$XDG_CACHE_HOME/jax_llama_amd/tune_<arch>.json``), loaded at first use and
rewritten after every new measurement, so a later process skips the measurement (a cold B = 8 prefill
autotunes for ~1 s).
"""
from __future__ import annotations

import contextlib
import json
import os
from typing import Dict, Optional, Tuple

import torch

_CACHE: Dict[Tuple, int] = {}
ENABLED = os.environ.get("JLA_AUTOTUNE", "1") != "0"
ARCH = "gfx950"

# ---- TP scope: the comm whose rank 0 decides (None: every process decides for itself)
_SCOPE = {"comm": None}


@contextlib.contextmanager
def tp_scope(comm):
    """Decisions taken inside are made by rank 0 of ``comm`` (when it spans > 1 rank) and broadcast."""
    prev = _SCOPE["comm"]
    _SCOPE["comm"] = comm if comm is not None and getattr(comm, "size", 1) > 1 else None
    try:
        yield
    finally:
        _SCOPE["comm"] = prev


def _collective(decide):
    """Run ``decide()`` on rank 0 of the current TP scope and broadcast its (JSON-able) result."""
    comm = _SCOPE["comm"]
    if comm is None or comm.group is None and not _dist_ready():
        return decide()
    import torch.distributed as dist
    obj = [decide() if comm.rank == 0 else None]
    src = dist.get_global_rank(comm.group, 0) if comm.group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=comm.group)
    v = obj[0]
    return tuple(v) if isinstance(v, list) else v


def _dist_ready() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


# ---- persistence
_LOADED = {"done": False}


def tune_file() -> str:
    env = os.environ.get("JLA_TUNE_FILE")
    if env:
        return env
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "jax_llama_amd", f"tune_{ARCH}.json")


TUNE_VERSION = 12  # bumped when a candidate set changes (2: split-K GEMV 16-19; 3: 4-tile split-K 26; 4: gemm4 tile 7; 5: gemm4 stream-K; 6: never-picked GEMV variants removed; 7: gemm4 256 x 128 tiles; 8: gemm5 tiles 11 / 12; 9: gemm4 rasterised in groups of 4 m-tiles; 10: stream-K / hybrid plans replaced by the exchange split; 11: gemm4 with the weights three K-tiles deep, 256 x 192 tiles; 12: the never-picked tiles 8 / 10 / 15 removed), so older persisted picks are re-measured


def _key_str(kind: str, key: Tuple) -> str:
    return f"{kind}@{TUNE_VERSION}:" + ",".join(str(k).replace("torch.", "") for k in key)


# The packaged table: picks measured on an MI355X with tools/bench_full.sh (JLA_TUNE_FILE) for the bench / latency /
# tensor-parallel shapes, shipped with the package so every box runs the same plans (the tuner's interleaved minimum
# flips between near-tied plans from box to box) and skips the first-use measurements. The user's file overrides it;
# JLA_TUNE_PACKAGED=0 ignores it (every shape measured on this device).
PACKAGED_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"tune_{ARCH}.json")


def _read_table(path: str) -> Dict[str, object]:
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        return {}
    return data if isinstance(data, dict) else {}


def _load():
    if _LOADED["done"]:
        return
    _LOADED["done"] = True
    if not _persist_on():
        return
    if os.environ.get("JLA_TUNE_PACKAGED", "1") != "0":
        _PERSISTED.update(_read_table(PACKAGED_FILE))
    _PERSISTED.update(_read_table(tune_file()))


_PERSISTED: Dict[str, object] = {}


def _persist_on() -> bool:
    """Picks are persisted unless disabled, or unless the candidate set is restricted for an A/B run (JLA_TUNE_TILES):
    a pick among a subset must never be reused by a run that searches the whole set."""
    return os.environ.get("JLA_TUNE_PERSIST", "1") != "0" and not os.environ.get("JLA_TUNE_TILES")


def _save(kind: str, key: Tuple, value):
    if not _persist_on():
        return
    _PERSISTED[_key_str(kind, key)] = list(value) if isinstance(value, tuple) else value
    path = tune_file()
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(_PERSISTED, f, indent=0, sort_keys=True)
        os.replace(tmp, path)
    except OSError:
        pass


def _persisted(kind: str, key: Tuple) -> Optional[object]:
    _load()
    v = _PERSISTED.get(_key_str(kind, key))
    return tuple(v) if isinstance(v, list) else v


def m_bucket(m: int) -> int:
    return 1 if m == 1 else (16 if m <= 16 else (32 if m <= 32 else 64))


def heuristic(m: int, n: int, k: int, mode: int) -> int:
    """Static choice from MI355X measurements (Llama-3-8B projections, profiles/README.md)."""
    ntt = n // 16
    if m > 16:
        return 6 if n % 32 == 0 else 1
    if m <= 4:
        return 1
    if ntt // 4 >= 384 and n % 64 == 0:
        return 5
    if ntt // 2 >= 192:
        return 6
    return 1


def candidates(m: int, n: int, swiglu: bool = False, bf16_x: bool = True) -> Tuple[int, ...]:
    # M > 16: two or four activation m-tiles per weight fragment, so the 2/4-tile GEMV workgroups
    # (fewer activation re-reads) and the tiled MFMA GEMM win on some shapes (M=24..64 sweep,
    # profiles/r1_decode_m32_variants.jsonl: qkv -> 6, gate_up -> 5, down/lm_head -> 7 at M=32)
    c = [1, 6]
    if n % 64 == 0:
        c.insert(1, 5)
    if m > 16:
        c.append(TILED_VARIANT)
        if bf16_x:
            # doubled hand-counted ring (4 waves, 2 tiles): at M > 16 the single ring keeps only 2 k-steps in flight
            # per wave (profiles/r2_decode_m32_asm_ring.jsonl)
            c.append(10)
    if n // 32 < 512:
        c.append(20)  # 2 tiles x 8 waves: few column groups (w1|w3 shards)
    if bf16_x and n // 16 <= SPLIT_MAX_GROUPS:
        # split-K GEMV (K over 2 workgroups per column group, in-kernel last-arriver sum): few column groups
        c.append(16)
    return tuple(c)


SPLIT_MAX_GROUPS = 1024  # csrc GEMV_SPLIT_MAX_GROUPS
SPLIT_GEMV = (16, 18, 26)  # split-K GEMV variants (gemv.hip gemv_split_variant)


TILED_VARIANT = 7


XP_CANDIDATES = (12, 15, 18, 21, 22, 26)  # packed-x GEMV variants (gemv.hip dispatch_nt; 18 / 26 split-K)


def choose(e, x: torch.Tensor, w, mode: int, run, xp_in: bool = False, pack_out: bool = False,
           no_split: bool = False, tiled_packs: bool = False) -> int:
    """``run(variant, x, weight_tensor)`` launches the op once. ``xp_in``: a packed copy of x exists, so the
    packed-x variants compete too; ``pack_out``: the epilogue must also write a packed copy of its output,
    which the GEMV variants do, and the tiled GEMM when ``tiled_packs`` (its split-K plan); ``no_split``: without the split-K GEMV
    variants (16 / 18 / 26; the fused-argmax lm_head GEMV has no split form)."""
    m = x.shape[0]
    # (TP-scoped decisions are cached apart: every rank of the group must take the same collective path)
    key = (m_bucket(m), w.n, w.k, mode, x.dtype, xp_in, pack_out, no_split, tiled_packs, _SCOPE["comm"] is not None)
    v = _CACHE.get(key)
    if v is not None:
        return v
    cands = list(candidates(m, w.n, swiglu=(mode == 2), bf16_x=(x.dtype == torch.bfloat16)))
    if pack_out:  # the tiled GEMM qualifies when its split-K reduce epilogue writes the copy (``tiled_packs``)
        cands = [c for c in cands if c != TILED_VARIANT or tiled_packs]
    if xp_in and x.dtype == torch.bfloat16:
        cands += [c for c in XP_CANDIDATES if (mode != 2 or c != 12) and
                  (c != 18 or w.n // 16 <= SPLIT_MAX_GROUPS) and (c != 21 or w.n // 32 < 512) and
                  (c != 22 or (w.n % 64 == 0 and w.n // 64 >= 64)) and
                  # 4-tile split-K: narrow outputs only (few 64-column groups), M > 16
                  (c != 26 or (m > 16 and w.n % 64 == 0 and w.n // 64 < 256))]
    if no_split:
        cands = [c for c in cands if c not in SPLIT_GEMV]
    if not ENABLED or torch.cuda.is_current_stream_capturing():
        h = heuristic(m, w.n, w.k, mode)
        return h if h in cands else 1
    def decide():
        pv = _persisted("gemv", key[:-1])
        if pv in cands:
            return pv
        mv = _measure(x, w, run, tuple(cands))
        _save("gemv", key[:-1], mv)
        return mv

    v = _collective(decide)
    _CACHE[key] = v
    return v


def _measure(x, w, run, cands) -> int:
    """Time every candidate on rotating scratch weights (> the Infinity Cache, so each call streams from HBM).
    Decode GEMVs take 3-20 us, below the host's launch rate, so eager back-to-back calls would time the host: the
    calls are captured into one hipGraph per candidate and the graph replay is timed (as the decode step runs them)."""
    nbytes = w.weight.numel() * 2
    copies = max(2, min(16, (640 << 20) // max(nbytes, 1) + 1))
    ws = [torch.empty_like(w.weight).normal_(0, 0.02) for _ in range(copies)]
    for v in cands:  # warm-up: code objects, workspaces (nothing may be allocated under capture)
        for i in range(2):
            run(v, x, ws[i % copies])
    torch.cuda.synchronize()
    iters = 2 * copies
    graphs = {}
    for v in cands:
        if v == TILED_VARIANT:  # its plan (and workspace) is chosen per call: timed eagerly (a long kernel anyway)
            graphs[v] = None
            continue
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                for i in range(iters):
                    run(v, x, ws[i % copies])
            graphs[v] = g
        except RuntimeError:  # a candidate that cannot be captured is timed eagerly
            graphs[v] = None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {v: float("inf") for v in cands}
    for _ in range(TUNE_ROUNDS):  # interleaved rounds, min per candidate (see _measure_plan)
        for v in cands:
            g = graphs[v]
            ev0.record()
            if g is not None:
                g.replay()
            else:
                for i in range(iters):
                    run(v, x, ws[i % copies])
            ev1.record()
            ev1.synchronize()
            times[v] = min(times[v], ev0.elapsed_time(ev1) / iters)
    del ws, graphs
    _TIMES[(x.shape[0], w.n, w.k, len(_TIMES))] = {v: round(t * 1000.0, 2) for v, t in times.items()}
    return min(cands, key=times.get)


_TIMES: Dict[Tuple, Dict[int, float]] = {}  # (m, n, k, seq) -> {variant: us per call} of every measured GEMV choice


def table() -> Dict[Tuple, int]:
    return dict(_CACHE)


def measured() -> Dict[Tuple, Dict[int, float]]:
    """Graph-timed microseconds per candidate of every GEMV choice measured in this process (tools/decode_point.py
    --tune-report)."""
    return dict(_TIMES)


# ----------------------------------------------------------------------------------------------
# Split-K factor of the tiled GEMM (csrc/kernels/gemm.hip) for decode-sized M: more K splits fill
# more CUs but every split writes and re-reads an fp32 [M, N] slab, so the best factor depends on
# (M, N, K) -- at M=256 it measured 8 for qkv/o (K=4096), 16 for down (K=14336), 2 for gate_up
# (profiles/README.md). Timed once per shape when the library heuristic asks for a split.
_KS_CACHE: Dict[Tuple, Tuple[int, int]] = {}
KS_CANDIDATES = (1, 2, 3, 4, 6, 8, 12, 16)
# tile configs: 1 / 2 / 3 gemm2 256x256, 128x256, 128x128 (csrc/kernels/gemm.hip tile_cfg); 7 gemm4; 14 gemm4 with the
# weights three K-tiles deep (160 KiB of LDS); 17 / 16 gemm4 on 256 x 128 / 192 tiles with the deep weights (no K split
# under the fused norm, its statistic is precomputed); 11 / 12: gemm5, the weight-streaming split-K kernel (gemm5ws.h;
# 256 / 128 columns per workgroup, M <= 256 per tile). What the bench shapes pick (BENCH_r05 gemm_plan_choice):
#   Llama-3-8B M = 1024 / 2048: qkv 16 / 17, o 17, gate_up 7 / 14 / 16, down 14 / 17 (split 2), lm_head 14;
#   Llama-3-70B M = 256 (MP 1 and the MP 8 shard): 1 / 3 (split 4 / 12), 11 / 12 (gemm5 splits), 14, 17.
TILE_CANDIDATES = (1, 2, 3, 7, 11, 12, 14, 16, 17)
if os.environ.get("JLA_TUNE_TILES"):  # A/B tooling: restrict the tile candidates, e.g. JLA_TUNE_TILES=1,2,3,7,11,12
    TILE_CANDIDATES = tuple(int(v) for v in os.environ["JLA_TUNE_TILES"].split(","))
# decode-sized M measured per shape (above: the C++ heuristic; prefill-sized M have enough 256 x 256 tiles)
TUNE_MAX_M = int(os.environ.get("JLA_TUNE_MAX_M", "4096"))


def choose_gemm_plan(e, m: int, n: int, k: int, device, mode: int = 0, rms: bool = False) -> Tuple[int, int]:
    """(split-K factor, gemm2 tile config) for this shape and epilogue: measured once on the device for
    decode-sized M (every tile config x every split that keeps >= 4 K-tiles per split); the C++ heuristic
    otherwise or while a hipGraph is being captured. The epilogue is part of the key: a split plan pays it
    in the reduce kernel, and the residual epilogue (fp32 read-modify-write + bf16 mirror) costs the reduce
    ~2x the bf16 store's, which moves the best split factor of wo / w2."""
    mode = 0 if mode == 3 else mode  # QKV (RoPE + cache write, side effects) is tuned as a plain store
    key = (m, n, k, mode, bool(rms), _SCOPE["comm"] is not None)
    plan = _KS_CACHE.get(key)
    if plan is not None:
        return plan
    heur = e.gemm_ksplit(m, n, k)
    # tuned band: decode-sized M (prefill-sized M has enough 256x256 tiles; tuning it would also need
    # multi-GB scratch outputs)
    if m <= 128 or m > TUNE_MAX_M or not ENABLED or device.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return heur, 0
    def decide():
        pv = _persisted("gemm", key[:-1])
        if isinstance(pv, tuple) and len(pv) == 2:
            return pv
        mv = _measure_plan(e, m, n, k, device, heur, mode, rms)
        _save("gemm", key[:-1], mv)
        return mv

    plan = tuple(_collective(decide))
    _KS_CACHE[key] = plan
    return plan


def choose_gemm_ksplit(e, m: int, n: int, k: int, device) -> int:
    return choose_gemm_plan(e, m, n, k, device)[0]


G4N_TILES = (16, 17)  # gemm4 on 256 x 192 / 128 tiles (csrc/kernels/gemm4w.h g4n_mainloop, deep weights)
G5_TILES = (11, 12)  # gemm5 weight-streaming split-K (csrc/kernels/gemm5ws.h)
TUNE_ROUNDS = 3


# split-K candidates whose fp32 partial slabs (split x M x N) exceed this are not measured: a K split only pays where the
# output has too few tiles, i.e. small M x N, and the scratch of a split lm_head at M = 4096 would be tens of GB
TUNE_WS_BYTES = int(float(os.environ.get("JLA_TUNE_WS_GB", "4")) * (1 << 30))


def _measure_plan(e, m, n, k, device, heur, mode=0, rms=False) -> Tuple[int, int]:
    kt = k // 32

    def fits(c):
        return c * m * (n + 1) * 4 <= TUNE_WS_BYTES

    ks_c = sorted({c for c in KS_CANDIDATES if kt // c >= 4 and fits(c)} | ({heur} if fits(heur) else set()) | {1})
    cands = [(c, tm) for tm in TILE_CANDIDATES for c in ks_c
             if (tm not in G4N_TILES or (k % 64 == 0 and not (c > 1 and rms and mode != 1)))
             and (tm not in G5_TILES or (k % 64 == 0 and m <= 512))]
    if k % 64 == 0 and m <= 512:  # gemm5 also at the deeper splits its 64-deep stages allow (narrow shards, long K)
        cands += [(c, tm) for tm in G5_TILES for c in (24, 32, 48) if (k // 64) // c >= 2 and c not in ks_c and fits(c)]
    nbytes = n * k * 2
    copies = max(2, min(16, (640 << 20) // max(nbytes, 1) + 1))
    ws_w = [torch.empty(n // 16, k // 32, 64, 8, dtype=torch.bfloat16, device=device).normal_(0, 0.02)
            for _ in range(copies)]
    x = torch.randn(m, k, device=device).to(torch.bfloat16)
    # the real epilogue's output: residual (fp32 in-place + bf16 mirror), SwiGLU (N/2 bf16), store (bf16)
    mirror = None
    if mode == 1:
        out = torch.zeros(m, n, dtype=torch.float32, device=device)
        mirror = torch.empty(m, n, dtype=torch.bfloat16, device=device)
    else:
        out = torch.empty(m, n // 2 if mode == 2 else n, dtype=torch.bfloat16, device=device)
    eps = 1e-5 if (rms and mode != 1) else -1.0
    need = max(c for c, _ in cands) * m * (n + 1)
    ws = torch.empty(need, dtype=torch.float32, device=device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rms_ws = torch.empty(m, dtype=torch.float32, device=device)  # as ops._rms_ws: the statistic ahead of gemm4

    def run(c, tm, i):
        if tm in G5_TILES:
            e.gemm(x, ws_w[i % copies], n, k, out, mode, True, mirror, c, ws, eps, tm)
        else:
            e.gemm(x, ws_w[i % copies], n, k, out, mode, True, mirror, c, ws if c > 1 else None, eps, tm,
                   None, rms_ws if c == 1 and eps > 0 else None)

    for c, tm in cands:  # warm every variant (code objects, caches) before any timing
        for i in range(2):
            run(c, tm, i)
    # interleaved rounds, min per candidate: one round alone is at the mercy of DVFS drift between
    # candidates (cdna_hip_programming.md rule 24)
    times = {cand: float("inf") for cand in cands}
    iters = 2 * copies
    for _ in range(TUNE_ROUNDS):
        for c, tm in cands:
            ev0.record()
            for i in range(iters):
                run(c, tm, i)
            ev1.record()
            ev1.synchronize()
            times[(c, tm)] = min(times[(c, tm)], ev0.elapsed_time(ev1) / iters)
    best = min(cands, key=times.get)
    del ws_w, ws
    return best


def ksplit_table() -> Dict[Tuple, int]:
    return dict(_KS_CACHE)


def variant_table() -> Dict[str, int]:
    """The decode-kernel variant picked per (M bucket, N, K, mode, ...) shape so far (bench.py reports it: which
    variants production shapes actually use)."""
    return {f"m{k[0]}_n{k[1]}_k{k[2]}_mode{k[3]}" + ("_xp" if k[5] else "") + ("_pack" if k[6] else "") +
            ("_nosplit" if k[7] else "") + ("_tp" if k[9] else ""): v for k, v in _CACHE.items()}
