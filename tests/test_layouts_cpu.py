"""CPU checks of the host-side layout and selection logic behind the decode kernels: the packed activation layout
(csrc/kernels/common.h pack_off, ops/reference.py pack_act) and the autotuner's candidate sets for the packed-x
variants (ops/autotune.py)."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd import ops
from jax_llama_amd.ops import autotune
from jax_llama_amd.ops import reference as ref


def pack_off(m: int, k: int, K: int) -> int:
    """Python mirror of common.h pack_off."""
    return (((m >> 4) * (K >> 5) + (k >> 5)) * 64 + (m & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7)


@pytest.mark.parametrize("m,k", [(1, 32), (12, 256), (16, 4096), (20, 96), (40, 128)])
def test_pack_act_matches_kernel_offsets_and_roundtrips(m, k):
    x = torch.arange(m * k, dtype=torch.float32).reshape(m, k)
    rows = ops.packed_rows(m)
    p = ref.pack_act(x, rows).reshape(-1)
    for mm in range(m):
        for kk in range(k):
            assert p[pack_off(mm, kk, k)].item() == x[mm, kk].item()
    assert torch.equal(ref.unpack_act(ref.pack_act(x, rows), m), x)
    # padding rows are zero in the reference copy (the kernels never read them into stored outputs)
    assert p.numel() == rows * k


def test_packed_rows_match_gemv_m_tiles():
    assert [ops.packed_rows(m) for m in (1, 16, 17, 32, 33, 64)] == [16, 16, 32, 32, 64, 64]


class _W:
    def __init__(self, n, k):
        self.n, self.k = n, k


@pytest.mark.parametrize("m", [12, 24, 40])
def test_autotune_candidates_for_packed_modes(m, monkeypatch):
    """Without measurements (autotune off / under capture) the choice must still respect the packed-mode rules:
    a required packed output excludes the tiled (7) kernel; SwiGLU never gets the one-tile packed-x variant (12)."""
    monkeypatch.setattr(autotune, "ENABLED", False)
    autotune._CACHE.clear()
    x = torch.zeros(m, 4096, dtype=torch.bfloat16)
    for n, mode in ((6144, 3), (4096, 1), (28672, 2), (4096, 0)):
        v = autotune.choose(None, x, _W(n, 4096), mode, run=None, xp_in=True, pack_out=True)
        assert v not in (4, autotune.TILED_VARIANT), (n, mode, v)
        if mode == 2:
            assert v not in (12, 14)


def test_pinned_variant_respects_packed_rules(monkeypatch):
    """ops._variant with a pinned GEMV variant: packed-x variants fall back when no packed x exists, SwiGLU maps
    12 to the two-tile 15, a required packed output never lands on the tiled GEMM (7)."""
    x = torch.zeros(20, 4096, dtype=torch.bfloat16)
    w = _W(28672, 4096)
    cases = [(12, None, None, ops.MODE_STORE, 1), (12, x, None, ops.MODE_STORE, 12), (12, x, None, ops.MODE_SWIGLU, 15),
             (15, x, x, ops.MODE_SWIGLU, 15), (7, None, x, ops.MODE_RESIDUAL, 1), (10, None, None, ops.MODE_STORE, 10)]
    for pinned, xp, po, mode, want in cases:
        monkeypatch.setattr(ops, "GEMV_VARIANT", pinned)
        assert ops._variant(None, x, w, mode, xp, po) == want, (pinned, mode)


def test_packaged_tune_table_is_current():
    """The shipped picks (ops/tune_gfx950.json, measured on an MI355X by tools/bench_full.sh) are keyed at the current
    TUNE_VERSION and name only plans the tuner could pick today: tile configs of TILE_CANDIDATES (or the gemm5 deep
    splits) and GEMV variants of the candidate lists -- a candidate-set change without a new table fails here."""
    import json
    from jax_llama_amd.ops import autotune
    with open(autotune.PACKAGED_FILE) as f:
        table = json.load(f)
    assert table, "empty packaged table"
    gemv_ok = {1, 5, 6, 10, 16, 20, autotune.TILED_VARIANT, *autotune.XP_CANDIDATES}
    for key, v in table.items():
        kind, rest = key.split("@", 1)
        assert int(rest.split(":", 1)[0]) == autotune.TUNE_VERSION, key
        if kind == "gemm":
            ks, tile = v
            assert tile in autotune.TILE_CANDIDATES and ks >= 1, (key, v)
        else:
            assert kind == "gemv" and v in gemv_ok, (key, v)
