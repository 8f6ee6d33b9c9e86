"""gemm4 -- the 4-wave 256 x 256 GEMM (one wave per SIMD, 128 x 128 AGPR accumulators per wave, 64-deep K-tiles;
csrc/kernels/gemm4w.h) -- against the pure-PyTorch fp32 reference and against gemm2 (tile config 1) for every
epilogue: bf16 / fp32 store, SwiGLU, residual + mirror, the RoPE / KV-cache write, the fused argmax; with and
without the fused RMSNorm statistic; data-parallel and split-K (partial slabs + reduce kernel); ragged M and N.
Reference ops: jax_llama/model.py:210, :294, :338, :736."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd import ops
from jax_llama_amd.models.weights import PackedLinear
from jax_llama_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16 = torch.bfloat16
G4 = 7  # tile config of gemm4 (csrc/kernels/gemm.hip G4_TILE)


def _close(a, b, rtol, atol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= atol + rtol * scale, f"max err {err:.3e} (ref max {scale:.3e})"


def _run_all(e, xg, pg, gp, h0, n, k, ks, ws, tile, rms_ws=None):
    """rms_ws: the fused norm's row statistic computed ahead of the GEMM (gemm4 without a K split)."""
    outs = []
    for eps in (-1.0, 1e-5):
        rw = rms_ws if eps > 0 else None
        o = torch.empty(xg.shape[0], n, dtype=torch.float32, device=DEV)
        e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, ks, ws, eps, tile, None, rw)
        ob = torch.empty(xg.shape[0], n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, ob, ops.MODE_STORE, True, None, ks, ws, eps, tile, None, rw)
        o2 = torch.empty(xg.shape[0], n // 2, dtype=BF16, device=DEV)
        e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, ws, eps, tile, None, rw)
        outs += [o, ob, o2]
    hg, mir = h0.clone(), torch.empty(h0.shape, dtype=BF16, device=DEV)
    e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws, -1.0, tile)
    torch.cuda.synchronize()
    return outs + [hg, mir]


@pytest.mark.parametrize("m,n,k,ks", [(200, 768, 1024, 1), (512, 1056, 1024, 1), (700, 2560, 4096, 1),
                                      (300, 768, 2048, 3), (2048, 4096, 4096, 2), (1000, 6144, 1536, 1),
                                      (256, 512, 128, 1), (300, 768, 192, 3)])
def test_gemm4_every_epilogue(m, n, k, ks):
    e = ops.ext()
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
    gp = PackedLinear.from_dense(gu, DEV)
    xg = x.to(DEV)
    h0 = torch.randn(m, n).to(DEV)
    ws = torch.empty(ks * m * (n + 1), dtype=torch.float32, device=DEV) if ks > 1 else None
    g4 = _run_all(e, xg, pg, gp, h0, n, k, ks, ws, G4)
    again = _run_all(e, xg, pg, gp, h0, n, k, ks, ws, G4)
    g2 = _run_all(e, xg, pg, gp, h0, n, k, ks, ws, 1)
    for i, (a, b) in enumerate(zip(g4, again)):
        assert torch.equal(a, b), f"output {i}: not reproducible"
    # vs gemm2: the same MFMA products in the same K order per output element; the row statistic of the fused norm
    # is summed in the same order, so the outputs agree to the last bit or within one rounding of bf16 outputs
    for i, (a, b) in enumerate(zip(g4, g2)):
        _close(a, b, 1e-2, 1e-3)
    _close(g4[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)
    _close(g4[1], ref.linear(x, w, None, torch.float32), 2e-2, 2e-2)
    _close(g4[3], ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)
    _close(g4[2], ref.linear_swiglu(x, gu, None), 3e-2, 3e-2)
    _close(g4[5], ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
    _close(g4[6], ref.linear_residual(x, w, h0.cpu().clone()), 1e-2, 1e-3)
    torch.testing.assert_close(g4[7].cpu(), g4[6].cpu().to(BF16), rtol=0, atol=0)
    exact = [torch.equal(a, b) for a, b in zip(g4, g2)]
    print("bit-identical to gemm2:", exact)
    if ks == 1:  # the row statistic computed ahead of the GEMM (rms_rowinv): fp32-reference close, near the in-loop one
        pre = _run_all(e, xg, pg, gp, h0, n, k, ks, ws, G4, torch.empty(m, device=DEV))
        for i in (0, 1, 2, 6, 7):  # no norm: the same kernel
            assert torch.equal(pre[i], g4[i]), i
        _close(pre[3], ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)
        _close(pre[5], ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
        for i in (3, 4, 5):
            _close(pre[i], g4[i], 1e-2, 1e-3)


@pytest.mark.parametrize("m,s,n_heads", [(512, 512, 8), (256, 1, 32), (300, 3, 8)])
def test_gemm4_qkv_rope_epilogue(m, s, n_heads):
    """The RoPE / KV-cache write in gemm4's epilogue (rotation in fp32 on the lane's two column pairs) against the
    fp32 oracle and gemm2's LDS-staged epilogue."""
    e = ops.ext()
    hkv, dh, k, t = 8, 128, 4096, 600
    h = n_heads
    b = m // s
    n = (h + 2 * hkv) * dh
    assert e.gemm_qkv_direct_ok(m, G4, k)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(BF16)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.randint(0, 1000, (m,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.linear_qkv_rope(x.float(), w, 1e-5, table, pos, kc, vc, 11, s, h, hkv, dh)
    pg = PackedLinear.from_dense(w, DEV)
    outs = {}
    for tile in (G4, 1):
        kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
        qg = torch.empty(m, h, dh, dtype=BF16, device=DEV)
        e.gemm_qkv(x.to(DEV), pg.weight, n, k, table.to(DEV), pos.to(DEV), kg, vg,
                   torch.tensor([11], dtype=torch.int32, device=DEV), s, h, hkv, dh, qg, 1, None, 1e-5, tile,
                   torch.empty(m, device=DEV) if tile == G4 else None)
        outs[tile] = (qg.cpu(), kg.cpu(), vg.cpu())
    qg, kg, vg = outs[G4]
    _close(qg, q, 2e-2, 2e-2)
    _close(kg, kc, 2e-2, 2e-2)
    _close(vg, vc, 2e-2, 2e-2)
    for a, c in zip(outs[G4], outs[1]):
        _close(a, c, 1e-2, 1e-2)


@pytest.mark.parametrize("m,n,k", [(256, 1008, 512), (300, 4096, 1024), (700, 2560, 1024)])
def test_gemm4_argmax(m, n, k):
    """gemm_argmax on gemm4 (2 partials per 256-column tile): exactly the stored-logits argmax (index and value),
    planted exact ties included."""
    e = ops.ext()
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    for src, dst in ((3, 700 % n), (17, 18), (n - 300, n - 1), (64, 63), (100, 200)):
        w[src] = (w[src].float() * 8).to(BF16)
        w[dst] = w[src]
    pg = PackedLinear.from_dense(w, DEV)
    xg = x.to(DEV)
    try:
        e.gemm_set_g4_default(1)
        for eps in (-1.0, 1e-5):
            logits = torch.empty(m, n, dtype=torch.float32, device=DEV)
            e.gemm(xg, pg.weight, n, k, logits, ops.MODE_STORE, True, None, 1, None, eps, G4)
            i0 = torch.empty(m, dtype=torch.int32, device=DEV)
            v0 = torch.empty(m, dtype=torch.float32, device=DEV)
            e.argmax(logits, i0, v0)
            ws = torch.empty(e.gemm_argmax_workspace(m, n), dtype=torch.float32, device=DEV)
            i1, v1 = torch.empty_like(i0), torch.empty_like(v0)
            e.gemm_argmax(xg, pg.weight, n, k, ws, eps, i1, v1)
            torch.cuda.synchronize()
            assert torch.equal(i0.cpu(), i1.cpu()), (eps, (i0 != i1).nonzero()[:8])
            assert torch.equal(v0.cpu(), v1.cpu())
            if eps > 0:  # the precomputed statistic: same as the stored-logits path with the same statistic
                rw = torch.empty(m, device=DEV)
                e.gemm(xg, pg.weight, n, k, logits, ops.MODE_STORE, True, None, 1, None, eps, G4, None, rw)
                e.argmax(logits, i0, v0)
                e.gemm_argmax(xg, pg.weight, n, k, ws, eps, i1, v1, rw)
                torch.cuda.synchronize()
                assert torch.equal(i0.cpu(), i1.cpu()) and torch.equal(v0.cpu(), v1.cpu())
    finally:
        e.gemm_set_g4_default(1)  # (the production default)


def test_gemm4_model_prefill_matches_gemm2():
    """A whole prefill (M = 2 x 160 rows: every projection on the tiled GEMM) with gemm4 as the tile-0 default vs
    gemm2: logits agree to bf16 rounding."""
    from helpers import gpu_config
    from jax_llama_amd.models import LLaMAForCausalLM
    e = ops.ext()
    cfg = gpu_config(hidden_size=512, intermediate_size=1536, num_attention_heads=4, num_key_value_heads=2,
                     vocab_size=1024)
    model = LLaMAForCausalLM(cfg, device=DEV, seed=0)
    toks = torch.randint(3, cfg.vocab_size, (2, 160), dtype=torch.int32)
    try:
        e.gemm_set_g4_default(0)
        base = model(toks).logits.float().cpu()
        e.gemm_set_g4_default(1)
        got = model(toks).logits.float().cpu()
    finally:
        e.gemm_set_g4_default(1)  # (the production default)
    _close(got, base, 2e-2, 2e-2)


@pytest.mark.parametrize("tile", [13, 14])
@pytest.mark.parametrize("m,n,k", [(2048, 4096, 1024), (700, 2560, 512), (4352, 1536, 256), (256, 1280, 192),
                                   (256, 2048, 128), (300, 1024, 64)])
def test_gemm4_persistent_identical(m, n, k, tile):
    """Tile configs 13 (persistent gemm4: one workgroup per CU over every tile) and 14 (the weight operand three
    K-tiles deep) run the same per-tile MFMA chain and epilogues as tile 7: store (fp32 / bf16), SwiGLU with the fused
    norm (precomputed / in-loop statistic) and the residual + mirror are bit-identical; ragged M / N, more tiles than
    CUs and every K-tile count of the deep ring's prologue / tail phases (1..4, 16) included."""
    e = ops.ext()
    torch.manual_seed(m + n + k + 13)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
    gp = PackedLinear.from_dense(gu, DEV)
    xg = x.to(DEV)
    h0 = torch.randn(m, n).to(DEV)
    rw = torch.empty(m, device=DEV)

    def run(tile):
        o = torch.empty(m, n, dtype=torch.float32, device=DEV)
        e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, 1, None, -1.0, tile)
        ob = torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, ob, ops.MODE_STORE, True, None, 1, None, 1e-5, tile, None, rw)
        o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
        e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, 1, None, 1e-5, tile, None, rw)
        o3 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
        e.gemm(xg, gp.weight, n, k, o3, ops.MODE_SWIGLU, True, None, 1, None, 1e-5, tile)
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, 1, None, -1.0, tile)
        torch.cuda.synchronize()
        return [o, ob, o2, o3, hg, mir]

    a, b = run(tile), run(G4)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), f"output {i}: tile {tile} differs from tile 7"
    _close(a[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)


@pytest.mark.parametrize("m,n,k,ks", [(256, 1280, 8192, 12), (256, 7168, 8192, 4), (512, 2048, 1024, 2),
                                      (256, 1024, 768, 3)])
def test_gemm4_deep_split_identical(m, n, k, ks):
    """The deep-W gemm4 (tile 14) under a K split (fp32 partial slabs + the reduce kernel, fused norm in-loop):
    bit-identical to tile 7 for the store and SwiGLU epilogues, and the residual epilogue, at the 70B shard's shapes."""
    e = ops.ext()
    torch.manual_seed(m + n + k + ks)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.02).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    xg = x.to(DEV)
    ws = torch.empty(ks * m * (n + 1), device=DEV)
    h0 = torch.randn(m, n).to(DEV)

    def run(tile):
        o = torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, ks, ws, 1e-5, tile)
        o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, ws, 1e-5, tile)
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws, -1.0, tile)
        torch.cuda.synchronize()
        return [o, o2, hg, mir]

    a, b = run(14), run(G4)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), f"output {i}: tile 14 differs from tile 7"
    xs = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    _close(a[0].float().cpu(), xs @ w.float().t(), 2e-2, 2e-2)


@pytest.mark.parametrize("tile", [16])
@pytest.mark.parametrize("m,n,k", [(2048, 6144, 512), (300, 1008, 256), (256, 4096, 128), (256, 1536, 192),
                                   (260, 768, 64)])
def test_gemm4_256x192_identical(m, n, k, tile):
    """256 x 192 tiles (tile 16, g4n_mainloop<6> with the weights three K-tiles deep): the same per-output MFMA
    chain as the 256 x 256 gemm4, so the store
    (fp32 / bf16, precomputed norm), SwiGLU, residual + mirror and split-K partial epilogues are bit-identical to tile 7;
    ragged N (a last tile narrower than 192 columns) included."""
    e = ops.ext()
    torch.manual_seed(m + n + k + 15)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    n2 = n // 32 * 32
    gp = PackedLinear.from_dense(ref.interleave_gate_up(w[: n2 // 2], w[n2 // 2: n2]), DEV)
    xg = x.to(DEV)
    h0 = torch.randn(m, n).to(DEV)
    rw = torch.empty(m, device=DEV)
    ws = torch.empty(2 * m * (n + 1), device=DEV)

    def run(tile):
        o = torch.empty(m, n, dtype=torch.float32, device=DEV)
        e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, 1, None, -1.0, tile)
        ob = torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, ob, ops.MODE_STORE, True, None, 1, None, 1e-5, tile, None, rw)
        o2 = torch.empty(m, n2 // 2, dtype=BF16, device=DEV)
        e.gemm(xg, gp.weight, n2, k, o2, ops.MODE_SWIGLU, True, None, 1, None, 1e-5, tile, None, rw)
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, 1, None, -1.0, tile)
        os = torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, os, ops.MODE_STORE, True, None, 2, ws, -1.0, tile)
        torch.cuda.synchronize()
        return [o, ob, o2, hg, mir, os]

    a, b = run(tile), run(G4)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), f"output {i}: tile {tile} differs from tile 7"
    _close(a[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)


@pytest.mark.parametrize("m,s", [(2048, 1), (512, 512), (300, 3)])
def test_gemm4_256x192_qkv_epilogue(m, s):
    """The RoPE / KV-cache write epilogue on 256 x 192 tiles (a tile spans 1.5 heads): q, K and V bit-identical to
    the 256 x 256 gemm4's."""
    e = ops.ext()
    h, hkv, dh, k = 32, 8, 128, 1024
    t = 11 + s + 4
    b = m // s
    n = (h + 2 * hkv) * dh
    assert e.gemm_qkv_direct_ok(m, 16, k)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(BF16)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.randint(0, 1000, (m,), dtype=torch.int32)
    pg = PackedLinear.from_dense(w, DEV)
    outs = {}
    for tile in (G4, 16):
        kg = torch.zeros(b, hkv, t, dh, dtype=BF16, device=DEV)
        vg = torch.zeros_like(kg)
        qg = torch.empty(m, h, dh, dtype=BF16, device=DEV)
        e.gemm_qkv(x.to(DEV), pg.weight, n, k, table.to(DEV), pos.to(DEV), kg, vg,
                   torch.tensor([11], dtype=torch.int32, device=DEV), s, h, hkv, dh, qg, 1, None, 1e-5, tile,
                   torch.empty(m, device=DEV))
        torch.cuda.synchronize()
        outs[tile] = (qg, kg, vg)
    for tile in (16,):
        for i, (u, v) in enumerate(zip(outs[tile], outs[G4])):
            assert torch.equal(u, v), f"qkv output {i}: tile {tile} differs from tile 7"


@pytest.mark.parametrize("tile", [17])
@pytest.mark.parametrize("m,n,k,ks", [(2048, 4096, 4096, 1), (700, 2560, 4096, 1), (300, 768, 2048, 2),
                                      (512, 1056, 1024, 1), (1000, 6144, 1536, 3), (256, 512, 128, 1),
                                      (256, 512, 192, 1), (256, 512, 64, 1)])
def test_gemm4_256x128_tiles(m, n, k, ks, tile):
    """Tile config 17 (gemm4 on 256 x 128 tiles, 4 n-tiles per wave, the weights three K-tiles deep): store
    (fp32 / bf16), SwiGLU, residual + mirror,
    split-K partials; the fused norm with its precomputed statistic. The same MFMA chain per output element as the
    256 x 256 gemm4 (tile 7), so bit-identical to it, and fp32-reference close; N not a multiple of 128 included."""
    e = ops.ext()
    torch.manual_seed(m + n + k + 10)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
    gp = PackedLinear.from_dense(gu, DEV)
    xg = x.to(DEV)
    h0 = torch.randn(m, n).to(DEV)
    ws = torch.empty(ks * m * (n + 1), dtype=torch.float32, device=DEV) if ks > 1 else None
    rw = torch.empty(m, device=DEV) if ks == 1 else None

    def run(tile):
        outs = []
        for eps in ((-1.0, 1e-5) if ks == 1 else (-1.0,)):
            r = rw if eps > 0 else None
            o = torch.empty(m, n, dtype=torch.float32, device=DEV)
            e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, ks, ws, eps, tile, None, r)
            ob = torch.empty(m, n, dtype=BF16, device=DEV)
            e.gemm(xg, pg.weight, n, k, ob, ops.MODE_STORE, True, None, ks, ws, eps, tile, None, r)
            o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
            e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, ws, eps, tile, None, r)
            outs += [o, ob, o2]
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws, -1.0, tile)
        torch.cuda.synchronize()
        return outs + [hg, mir]

    t10, t7 = run(tile), run(G4)
    for i, (a, b) in enumerate(zip(t10, t7)):
        assert torch.equal(a, b), f"output {i}: differs from the 256 x 256 gemm4"
    _close(t10[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)
    _close(t10[2], ref.linear_swiglu(x, gu, None), 3e-2, 3e-2)
    _close(t10[-2], ref.linear_residual(x, w, h0.cpu().clone()), 1e-2, 1e-3)
    torch.testing.assert_close(t10[-1].cpu(), t10[-2].cpu().to(BF16), rtol=0, atol=0)
    if ks == 1:
        _close(t10[3], ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)
        _close(t10[5], ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
