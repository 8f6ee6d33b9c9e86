"""gemm5 -- the weight-streaming split-K GEMM for decode batches of 128-256 rows (csrc/kernels/gemm5ws.h, tile
configs 11 / 12: each wave owns every row of the tile x 4 / 2 n-tiles and streams its packed weight fragments straight
into registers, x staged once per CU in LDS) -- against the pure-PyTorch fp32 reference for every epilogue the
reduce kernel runs: bf16 / fp32 store, SwiGLU, residual + mirror, the RoPE / KV-cache write; with and without the
fused RMSNorm statistic (summed by the kernel from the staged x); split counts that leave empty splits and ragged
stage counts; M above one 256-row tile; reproducible bit for bit.
Reference ops: jax_llama/model.py:210, :294, :338."""
from __future__ import annotations

import pytest
import torch

from jax_llama_amd import ops
from jax_llama_amd.models.weights import PackedLinear
from jax_llama_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16 = torch.bfloat16


def _close(a, b, rtol, atol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= atol + rtol * scale, f"max err {err:.3e} (ref max {scale:.3e})"


@pytest.mark.parametrize("tile", [11, 12])
@pytest.mark.parametrize("m,n,k,ks", [(256, 1280, 8192, 16), (256, 7168, 1024, 3), (200, 768, 1024, 1),
                                      (129, 512, 3584, 5), (100, 1024, 640, 2), (300, 2048, 1024, 4),
                                      (256, 512, 192, 7)])
def test_gemm5_every_epilogue(tile, m, n, k, ks):
    e = ops.ext()
    torch.manual_seed(m + n + k + tile)
    x = torch.randn(m, k).to(BF16)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
    gp = PackedLinear.from_dense(gu, DEV)
    xg = x.to(DEV)
    h0 = torch.randn(m, n).to(DEV)
    eks = e.gemm5_ksplit(k, ks)
    assert 1 <= eks <= ks
    ws = torch.empty(eks * m * (n + 1), dtype=torch.float32, device=DEV)

    def run():
        outs = []
        for eps in (-1.0, 1e-5):
            o = torch.empty(m, n, dtype=torch.float32, device=DEV)
            e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, ks, ws, eps, tile)
            ob = torch.empty(m, n, dtype=BF16, device=DEV)
            e.gemm(xg, pg.weight, n, k, ob, ops.MODE_STORE, True, None, ks, ws, eps, tile)
            o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
            e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, ws, eps, tile)
            outs += [o, ob, o2]
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws, -1.0, tile)
        torch.cuda.synchronize()
        return outs + [hg, mir]

    a, b = run(), run()
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), f"output {i}: not reproducible"
    _close(a[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)
    _close(a[1], ref.linear(x, w, None, torch.float32), 2e-2, 2e-2)
    _close(a[2], ref.linear_swiglu(x, gu, None), 3e-2, 3e-2)
    _close(a[3], ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)
    _close(a[5], ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
    _close(a[6], ref.linear_residual(x, w, h0.cpu().clone()), 1e-2, 1e-3)
    torch.testing.assert_close(a[7].cpu(), a[6].cpu().to(BF16), rtol=0, atol=0)


@pytest.mark.parametrize("tile", [11, 12])
@pytest.mark.parametrize("m,s,n_heads,hkv,ks", [(256, 1, 8, 1, 24), (200, 1, 32, 8, 4), (256, 2, 8, 2, 1)])
def test_gemm5_qkv_rope_epilogue(tile, m, s, n_heads, hkv, ks):
    """The RoPE / KV-cache write of the reduce kernel behind gemm5's partial slabs (Llama-3-70B MP 8 qkv shard: 8 q
    heads, 1 kv head) against the fp32 oracle."""
    e = ops.ext()
    dh, k, t = 128, 2048, 600
    h = n_heads
    b = m // s
    n = (h + 2 * hkv) * dh
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(BF16)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.randint(0, 1000, (m,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.linear_qkv_rope(x.float(), w, 1e-5, table, pos, kc, vc, 11, s, h, hkv, dh)
    pg = PackedLinear.from_dense(w, DEV)
    eks = e.gemm5_ksplit(k, ks)
    ws = torch.empty(eks * m * (n + 1), dtype=torch.float32, device=DEV)
    kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
    qg = torch.empty(m, h, dh, dtype=BF16, device=DEV)
    e.gemm_qkv(x.to(DEV), pg.weight, n, k, table.to(DEV), pos.to(DEV), kg, vg,
               torch.tensor([11], dtype=torch.int32, device=DEV), s, h, hkv, dh, qg, ks, ws, 1e-5, tile, None)
    torch.cuda.synchronize()
    _close(qg, q, 2e-2, 2e-2)
    _close(kg, kc, 2e-2, 2e-2)
    _close(vg, vc, 2e-2, 2e-2)
