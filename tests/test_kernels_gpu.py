"""Numerics of every gfx950 HIP kernel against the pure-PyTorch fp32 reference of the same op
(``jax_llama_amd/ops/reference.py``). GPU-only (``-m gpu``); the HIP path must be the one that runs:
``ops._ext.ext()`` raises if the extension is missing, it never falls back."""
from __future__ import annotations

import math

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


def test_extension_loaded():
    e = ops.ext()
    assert e.ARCH == "gfx950"
    assert e.__file__.startswith(__import__("os").path.dirname(__import__("jax_llama_amd").__file__))


def test_embedding():
    table = torch.randn(1000, 256, dtype=BF16)
    ids = torch.randint(0, 1000, (37,), dtype=torch.int32)
    out = ops.embedding(ids.to(DEV), table.to(DEV))
    torch.testing.assert_close(out.cpu(), ref.embedding(ids, table), rtol=0, atol=0)


@pytest.mark.parametrize("m,d", [(1, 4096), (7, 256), (130, 8192)])
def test_rms(m, d):
    x = torch.randn(m, d) * 3
    w = torch.randn(d)
    out = ops.rms_scale(x.to(DEV), 1e-5)
    _close(out, ref.rms_scale(x, 1e-5), 1e-2, 1e-2)
    out2 = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-5)
    _close(out2, ref.rmsnorm(x, w, 1e-5), 1e-5, 1e-4)


def _mk_linear(n, k, fold=None):
    w = (torch.randn(n, k) * 0.05).to(BF16)
    return w, PackedLinear.from_dense(w, DEV, fold=fold), PackedLinear.from_dense(w, "cpu", fold=fold)


def test_pack_roundtrip():
    w = torch.randn(64, 96).to(BF16)
    p = ref.pack_frag16x32(w)
    torch.testing.assert_close(ref.unpack_frag16x32(p, 64, 96), w, rtol=0, atol=0)


@pytest.mark.parametrize("m", [1, 5, 16, 17, 33, 64])
@pytest.mark.parametrize("n,k", [(256, 512), (48, 4096), (4096, 224)])
@pytest.mark.parametrize("rms", [False, True])
def test_linear_store(m, n, k, rms):
    x = torch.randn(m, k) * 2
    w, pg, pc = _mk_linear(n, k)
    eps = 1e-5 if rms else None
    y = ops.linear(x.to(DEV), pg, rms_eps=eps)
    _close(y, ops.linear(x, pc, rms_eps=eps), 2e-2, 2e-2)
    y32 = ops.linear(x.to(DEV), pg, rms_eps=eps, out_dtype=torch.float32)
    _close(y32, ref.linear(x, w, eps, torch.float32), 1e-2, 1e-3)


@pytest.mark.parametrize("m", [1, 16, 64, 65, 200])
def test_linear_residual_and_bf16_input(m):
    k, n = 1024, 512
    x = (torch.randn(m, k)).to(BF16)
    w, pg, pc = _mk_linear(n, k)
    h = torch.randn(m, n)
    hg = h.to(DEV)
    ops.linear_residual(x.to(DEV), pg, hg)
    _close(hg, ref.linear_residual(x, w, h.clone()), 1e-2, 1e-3)
    hg2 = h.to(DEV)
    ops.linear_residual(x.to(DEV), pg, hg2, accumulate=False)
    _close(hg2, ref.linear_residual(x, w, h.clone(), accumulate=False), 1e-2, 1e-3)


@pytest.mark.parametrize("m", [1, 3, 16, 40, 64, 100, 257])
@pytest.mark.parametrize("k", [512, 1376])
def test_linear_swiglu(m, k):
    f = 352
    w1 = (torch.randn(f, k) * 0.05).to(BF16)
    w3 = (torch.randn(f, k) * 0.05).to(BF16)
    gu = ref.interleave_gate_up(w1, w3)
    x = torch.randn(m, k)
    pg = PackedLinear.from_dense(gu, DEV)
    y = ops.linear_swiglu(x.to(DEV), pg, rms_eps=1e-5)
    g = ref.linear(x, w1, 1e-5, torch.float32)
    u = ref.linear(x, w3, 1e-5, torch.float32)
    expect = torch.nn.functional.silu(g) * u
    _close(y, expect, 3e-2, 3e-2)


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (300, 6144 // 8, 4096 // 8), (129, 1040, 96)])
def test_gemm_large_m(m, n, k):
    x = torch.randn(m, k)
    w, pg, pc = _mk_linear(n, k)
    y = ops.linear(x.to(DEV), pg, rms_eps=1e-6, out_dtype=torch.float32)
    xs = ref.rms_scale(x, 1e-6)
    expect = xs.float() @ w.float().t()
    _close(y, expect, 1e-2, 1e-3)


def test_rope_kv_write():
    b, s, h, hkv, dh, t = 3, 5, 8, 2, 128, 16
    qkv = torch.randn(b * s, (h + 2 * hkv) * dh).to(BF16)
    table = ref.rope_table(dh, 64, 10000.0)
    pos = torch.randint(-1, 40, (b * s,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.rope_kv_write(qkv, table, pos, kc, vc, 3, s, h, hkv, dh)
    kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
    slot = torch.tensor([3], dtype=torch.int32, device=DEV)
    qg = ops.rope_kv_write(qkv.to(DEV), table.to(DEV), pos.to(DEV), kg, vg, slot, s, h, hkv, dh)
    _close(qg, q, 1e-2, 1e-2)
    _close(kg, kc, 1e-2, 1e-2)
    torch.testing.assert_close(vg.cpu(), vc, rtol=0, atol=0)


def _cache(b, hkv, t, dh):
    return (torch.randn(b, hkv, t, dh) * 0.5).to(BF16), torch.randn(b, hkv, t, dh).to(BF16)


@pytest.mark.parametrize("rep", [1, 2, 4, 8])
@pytest.mark.parametrize("t,slot", [(40, 17), (300, 299), (1030, 700)])
def test_attention_decode(rep, t, slot):
    b, hkv, dh = 3, 2, 128
    h = hkv * rep
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, h, dh).to(BF16)
    kv_start = torch.tensor([0, 5, slot + 1], dtype=torch.int32)  # last row: no valid key -> zeros
    expect = ref.attention(q, kc, vc, slot, kv_start).reshape(b, h * dh)
    got = ops.attention(q.to(DEV), kc.to(DEV), vc.to(DEV), torch.tensor([slot], dtype=torch.int32, device=DEV),
                        kv_start.to(DEV))
    _close(got, expect, 2e-2, 2e-2)
    assert torch.isfinite(got.float()).all()
    assert got[2].float().abs().max().item() == 0.0


@pytest.mark.parametrize("rep", [1, 4, 8])
@pytest.mark.parametrize("t,slot", [(40, 17), (300, 299), (1030, 700)])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_decode_streaming_v2(rep, t, slot, masked):
    """The streaming (LDS-DMA ring, wave-per-item) decode kernel normally serves only large batches;
    force it at small B so its split + last-arriver merge path and the key-mask path are covered."""
    e = ops.ext()
    b, hkv, dh = 3, 2, 128
    h = hkv * rep
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, h, dh).to(BF16)
    kv_start = torch.tensor([0, 5, slot + 1], dtype=torch.int32)
    mask = None
    if masked:
        mask = (torch.rand(b, t) > 0.3).to(torch.uint8)
        mask[:, slot] = 1
    expect = ref.attention(q, kc, vc, slot, kv_start, mask).reshape(b, h * dh)
    try:
        e.attn_set_impl(2, -1)  # v2 for any batch size
        got = ops.attention(q.to(DEV), kc.to(DEV), vc.to(DEV), torch.tensor([slot], dtype=torch.int32, device=DEV),
                            kv_start.to(DEV), None if mask is None else mask.to(DEV))
        torch.cuda.synchronize()
    finally:
        e.attn_set_impl(2, 0)
    _close(got, expect, 2e-2, 2e-2)
    assert got[2].float().abs().max().item() == 0.0


@pytest.mark.parametrize("b", [512, 256, 128])
@pytest.mark.parametrize("rep", [1, 2, 4, 8])
@pytest.mark.parametrize("t,slot", [(300, 299), (520, 260)])
def test_attention_decode_v4_large_batch(rep, t, slot, b):
    """Large batch, one split, no key mask: the register-ring streaming kernel (v4) serves it (from 4096 (row, kv
    head) pairs, and mid-batch above 64 rows: every rep <= 4, rep 8 from 2048 pairs); compare with the fp32 reference
    and with the v2 LDS-DMA kernel (impl 4)."""
    e = ops.ext()
    hkv, dh = 8, 128
    h = hkv * rep
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, h, dh).to(BF16)
    g = torch.Generator().manual_seed(3)
    kv_start = torch.randint(0, slot // 2, (b,), generator=g, dtype=torch.int32)
    kv_start[7] = slot + 1  # a row with no valid key -> zeros
    expect = ref.attention(q, kc, vc, slot, kv_start).reshape(b, h * dh)
    args = (q.to(DEV), kc.to(DEV), vc.to(DEV), torch.tensor([slot], dtype=torch.int32, device=DEV), kv_start.to(DEV))
    assert e.attn_decode_splits(b, hkv, t, rep) == 1
    got = ops.attention(*args)
    try:
        e.attn_set_impl(4, 0)  # v2, (4-key group, 2 slots)
        got_v2 = ops.attention(*args)
        torch.cuda.synchronize()
    finally:
        e.attn_set_impl(2, 0)
    _close(got, expect, 2e-2, 2e-2)
    assert got[7].float().abs().max().item() == 0.0
    _close(got, got_v2, 1e-2, 1e-2)


def test_attention_decode_key_mask():
    b, hkv, rep, t, dh, slot = 2, 2, 4, 96, 128, 80
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, hkv * rep, dh).to(BF16)
    mask = (torch.rand(b, t) > 0.3).to(torch.uint8)
    mask[:, slot] = 1
    kv_start = torch.zeros(b, dtype=torch.int32)
    expect = ref.attention(q, kc, vc, slot, kv_start, mask).reshape(b, -1)
    got = ops.attention(q.to(DEV), kc.to(DEV), vc.to(DEV), torch.tensor([slot], dtype=torch.int32, device=DEV),
                        kv_start.to(DEV), mask.to(DEV))
    _close(got, expect, 2e-2, 2e-2)


@pytest.mark.parametrize("rep", [1, 4])
@pytest.mark.parametrize("s,slot0", [(7, 0), (64, 0), (130, 10)])
def test_attention_prefill(rep, s, slot0):
    b, hkv, dh = 2, 2, 128
    h = hkv * rep
    t = slot0 + s + 3
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, s, h, dh).to(BF16)
    kv_start = torch.tensor([0, min(slot0 + 4, slot0 + s - 1)], dtype=torch.int32)
    expect = ref.attention(q, kc, vc, slot0, kv_start).reshape(b * s, h * dh)
    got = ops.attention(q.to(DEV), kc.to(DEV), vc.to(DEV), torch.tensor([slot0], dtype=torch.int32, device=DEV),
                        kv_start.to(DEV))
    _close(got, expect, 2e-2, 2e-2)
    assert torch.isfinite(got.float()).all()


def _attn_ref_gpu(q, kc, vc, slot0, kv_start, key_mask=None, chunk=512):
    """fp32 PyTorch reference on the GPU (chunked over queries) for long sequences: query s of row b at
    slot slot0 + s attends keys j with kv_start[b] <= j <= slot0 + s (and key_mask[b, j])."""
    b, s, h, dh = q.shape
    hkv, t = kc.shape[1], kc.shape[2]
    rep = h // hkv
    k = kc.float().repeat_interleave(rep, 1)  # [B, H, T, Dh]
    v = vc.float().repeat_interleave(rep, 1)
    out = torch.empty(b, s, h, dh, device=q.device)
    j = torch.arange(t, device=q.device)
    for c0 in range(0, s, chunk):
        qc = q[:, c0:c0 + chunk].float().permute(0, 2, 1, 3)  # [B, H, c, Dh]
        sc = qc @ k.transpose(-1, -2) / dh ** 0.5
        qs = slot0 + c0 + torch.arange(qc.shape[2], device=q.device)
        ok = (j[None, None, :] <= qs[None, :, None]) & (j[None, None, :] >= kv_start[:, None, None])
        if key_mask is not None:
            ok = ok & (key_mask[:, None, :t] != 0)
        sc = sc.masked_fill(~ok[:, None], float("-inf"))
        p = torch.softmax(sc, -1).nan_to_num(0.0)
        out[:, c0:c0 + chunk] = (p @ v).permute(0, 2, 1, 3)
    return out.reshape(b * s, h * dh)


@pytest.mark.parametrize("impl", [2, 1, 7, 8, 9, 13])
@pytest.mark.parametrize("rep", [1, 4, 8])
@pytest.mark.parametrize("s,slot0,masked", [(7, 0, False), (130, 10, False), (512, 0, False), (300, 0, True),
                                            (2048, 0, False)])
def test_attention_prefill_long(impl, rep, s, slot0, masked):
    """Prefill attention at real prompt lengths (S up to 2048) with left padding (kv_start) or a general
    key mask, against an fp32 PyTorch reference; impl 2 = GQA-shared 32x32 MFMA kernel, 1 = v1."""
    e = ops.ext()
    if impl == 1 and s > 512:
        pytest.skip("v1 is the A/B baseline; long shapes covered by impl 2")
    b, hkv, dh = 2, 2, 128
    h = hkv * rep
    t = slot0 + s + 5
    g = torch.Generator(device=DEV).manual_seed(s * 10 + rep)
    kc = (torch.randn(b, hkv, t, dh, device=DEV, generator=g) * 0.5).to(BF16)
    vc = torch.randn(b, hkv, t, dh, device=DEV, generator=g).to(BF16)
    q = torch.randn(b, s, h, dh, device=DEV, generator=g).to(BF16)
    kv_start = torch.tensor([0, slot0 + s // 3], dtype=torch.int32, device=DEV)  # row 1 left-padded
    mask = None
    if masked:
        mask = (torch.rand(b, t, device=DEV, generator=g) > 0.3).to(torch.uint8)
        kv_start.zero_()
    slot = torch.tensor([slot0], dtype=torch.int32, device=DEV)
    try:
        e.attn_prefill_set_impl(impl)
        got = ops.attention(q, kc, vc, slot, kv_start, mask)
        torch.cuda.synchronize()
    finally:
        e.attn_prefill_set_impl(2)
    want = _attn_ref_gpu(q, kc, vc, slot0, kv_start, mask)
    assert torch.isfinite(got.float()).all()
    err = (got.float() - want).abs().max().item()
    assert err < 3e-2, err
    if not masked and s // 3 > 0:  # left-pad queries of row 1 (no valid key) output exactly 0
        assert got.reshape(b, s, h * dh)[1, : s // 3].float().abs().max().item() == 0.0


def test_attention_prefill_8k():
    """S = 8192 causal prefill (Llama-3 max_seq_len), rep 4, one batch row."""
    b, hkv, rep, s, dh = 1, 2, 4, 8192, 128
    h = hkv * rep
    g = torch.Generator(device=DEV).manual_seed(3)
    kc = (torch.randn(b, hkv, s, dh, device=DEV, generator=g) * 0.5).to(BF16)
    vc = torch.randn(b, hkv, s, dh, device=DEV, generator=g).to(BF16)
    q = torch.randn(b, s, h, dh, device=DEV, generator=g).to(BF16)
    kv_start = torch.zeros(b, dtype=torch.int32, device=DEV)
    got = ops.attention(q, kc, vc, torch.zeros(1, dtype=torch.int32, device=DEV), kv_start)
    want = _attn_ref_gpu(q, kc, vc, 0, kv_start, chunk=256)
    err = (got.float() - want).abs().max().item()
    assert err < 3e-2, err


@pytest.mark.parametrize("rep", [4, 8])
def test_attention_decode_8k(rep):
    """Decode attention over an 8192-slot cache (long context), left padding on one row."""
    b, hkv, t, dh = 2, 2, 8192, 128
    h = hkv * rep
    g = torch.Generator(device=DEV).manual_seed(rep)
    kc = (torch.randn(b, hkv, t, dh, device=DEV, generator=g) * 0.5).to(BF16)
    vc = torch.randn(b, hkv, t, dh, device=DEV, generator=g).to(BF16)
    q = torch.randn(b, 1, h, dh, device=DEV, generator=g).to(BF16)
    slot0 = t - 1
    kv_start = torch.tensor([0, 3000], dtype=torch.int32, device=DEV)
    got = ops.attention(q, kc, vc, torch.tensor([slot0], dtype=torch.int32, device=DEV), kv_start)
    want = _attn_ref_gpu(q, kc, vc, slot0, kv_start)
    err = (got.float() - want).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("m", [1, 5, 17, 40, 64])
@pytest.mark.parametrize("variant", [1, 5, 6, 10, 20])
def test_linear_skinny_argmax(m, variant):
    """Decode lm_head with the argmax in the GEMV epilogue == stored fp32 logits + first-max argmax,
    bit for bit (same accumulation order), including an exact tie across two 16-column tiles."""
    e = ops.ext()
    n, k = 2048, 512
    w = PackedLinear.random(n, k, DEV)
    x = torch.randn(m, k, device=DEV).to(BF16)
    logits = torch.empty(m, n, dtype=torch.float32, device=DEV)
    ws, tk = ops._skinny_ws(e, m, n, k, ops.MODE_STORE, x.device)
    e.linear_skinny(x, w.weight, n, k, logits, ops.MODE_STORE, 1e-5, True, variant, ws, tk)
    part = torch.empty(m * (n // 16) * 2, dtype=torch.float32, device=DEV)
    idx = torch.empty(m, dtype=torch.int32, device=DEV)
    val = torch.empty(m, dtype=torch.float32, device=DEV)
    e.linear_skinny_argmax(x, w.weight, n, k, 1e-5, variant, part, idx, val)
    want_v, want_i = logits.max(-1)
    assert torch.equal(idx.long().cpu(), logits.argmax(-1).cpu())
    assert torch.equal(val.cpu(), want_v.cpu())
    # tie: duplicate the weight rows of columns 100 and 900 -> equal logits, first index wins
    wd = w.dense().clone()
    wd[900] = wd[100]
    wt = PackedLinear.from_dense(wd.cpu(), DEV)
    xb = torch.zeros(m, k, device=DEV).to(BF16)
    xb[:, :] = wd[100].to(DEV)[None, :].to(BF16)  # makes column 100 (and 900) the maximum
    e.linear_skinny_argmax(xb, wt.weight, n, k, -1.0, variant, part, idx, val)
    assert idx.cpu().tolist() == [100] * m


def test_argmax_first_index():
    x = torch.randn(4, 128256)
    x[1, 77] = 100.0
    x[1, 9000] = 100.0  # tie: first index wins
    idx, val = ops.argmax(x.to(DEV))
    assert idx.cpu().tolist() == x.argmax(-1).tolist()
    assert idx[1].item() == 77
    torch.testing.assert_close(val.cpu(), x.max(-1).values)


@pytest.mark.parametrize("k,xdt", [(512, torch.float32), (256, BF16), (4096, BF16)])
@pytest.mark.parametrize("m,s", [(1, 1), (16, 1), (48, 1), (6, 3), (60, 20), (130, 65)])
def test_linear_qkv_rope_fused(m, s, k, xdt):
    """Also at the small K and bf16 activations of the GPU whole-model tests (hidden 256, bf16 mirror)."""
    h, hkv, dh, t = 4, 2, 128, 80
    b = m // s
    n = (h + 2 * hkv) * dh
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(xdt).float()
    table = ref.rope_table(dh, 256, 500000.0)
    pos = torch.randint(0, 200, (m,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.linear_qkv_rope(x, w, 1e-5, table, pos, kc, vc, 7, s, h, hkv, dh)
    kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
    pg = PackedLinear.from_dense(w, DEV)
    qg = ops.linear_qkv_rope(x.to(xdt).to(DEV), pg, 1e-5, table.to(DEV), pos.to(DEV), kg, vg,
                             torch.tensor([7], dtype=torch.int32, device=DEV), s, h, hkv, dh)
    _close(qg, q, 2e-2, 2e-2)
    _close(kg, kc, 2e-2, 2e-2)
    _close(vg, vc, 2e-2, 2e-2)


@pytest.mark.parametrize("variant", [16])
@pytest.mark.parametrize("m,s,k", [(1, 1, 8192), (16, 1, 4096), (32, 1, 8192), (64, 1, 1024), (6, 3, 256)])
def test_split_gemv_qkv_rope(m, s, k, variant):
    """Split-K GEMV (K over 2 workgroups per column group, last arriver sums + runs the epilogue): the fused
    qkv projection (RMS statistics summed over the splits, RoPE, KV-cache write) at tensor-parallel shard widths
    (10 heads = 80 column tiles, as Llama-3-70B at MP 8) against the fp32 oracle, and repeatable bit for bit (the
    tickets reset themselves)."""
    h, hkv, dh, t = 8, 1, 128, 80
    b = m // s
    n = (h + 2 * hkv) * dh
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(BF16).float()
    table = ref.rope_table(dh, 256, 500000.0)
    pos = torch.randint(0, 200, (m,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.linear_qkv_rope(x, w, 1e-5, table, pos, kc, vc, 7, s, h, hkv, dh)
    pg = PackedLinear.from_dense(w, DEV)
    ops.GEMV_VARIANT = variant
    try:
        outs = []
        for _ in range(3):
            kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
            qg = ops.linear_qkv_rope(x.to(BF16).to(DEV), pg, 1e-5, table.to(DEV), pos.to(DEV), kg, vg,
                                     torch.tensor([7], dtype=torch.int32, device=DEV), s, h, hkv, dh)
            outs.append((qg.cpu(), kg.cpu(), vg.cpu()))
    finally:
        ops.GEMV_VARIANT = 0
    qg, kg, vg = outs[0]
    _close(qg, q, 2e-2, 2e-2)
    _close(kg, kc, 2e-2, 2e-2)
    _close(vg, vc, 2e-2, 2e-2)
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0]))


def test_gemv_variants_agree():
    x = torch.randn(16, 2048, device=DEV)
    w = PackedLinear.from_dense((torch.randn(512, 2048) * 0.05).to(BF16), DEV)
    outs = []
    for v in (1, 5, 6, 16):
        ops.GEMV_VARIANT = v
        outs.append(ops.linear(x, w, rms_eps=1e-5, out_dtype=torch.float32))
    ops.GEMV_VARIANT = 0
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("k", [256, 4096])
@pytest.mark.parametrize("variant", [1, 5, 6, 10, 16, 20])
@pytest.mark.parametrize("m", [1, 9, 16, 40, 64])
def test_decode_linear_paths_all_modes(variant, m, k):
    """The decode GEMV's tile / ring-depth / split variants (at M > 16 the hand-counted doubled ring 10), every
    epilogue, real-ish K (multi-split) and the whole-model tests' K = 256."""
    ops.GEMV_VARIANT = variant
    try:
        n = 768
        x = torch.randn(m, k)
        w, pg, pc = _mk_linear(n, k)
        y = ops.linear(x.to(DEV), pg, rms_eps=1e-5, out_dtype=torch.float32)
        _close(y, ref.linear(x, w, 1e-5, torch.float32), 1e-2, 1e-3)
        xb = x.to(BF16)
        yb = ops.linear(xb.to(DEV), pg, rms_eps=1e-5, out_dtype=torch.float32)  # bf16 activations + fused norm
        _close(yb, ref.linear(xb.float(), w, 1e-5, torch.float32), 1e-2, 1e-3)
        h = torch.randn(m, n)
        hg = h.to(DEV)
        ops.linear_residual(xb.to(DEV), pg, hg)
        _close(hg, ref.linear_residual(xb, w, h.clone()), 1e-2, 1e-3)
        gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
        y2 = ops.linear_swiglu(x.to(DEV), PackedLinear.from_dense(gu, DEV), rms_eps=1e-5)
        _close(y2, ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
        # determinism of the split-K reduction (fixed order)
        y_again = ops.linear(x.to(DEV), pg, rms_eps=1e-5, out_dtype=torch.float32)
        assert torch.equal(y, y_again)
    finally:
        ops.GEMV_VARIANT = 0


@pytest.mark.parametrize("m", [40, 64, 96, 256])
def test_tiled_splitk_all_modes(m):
    """128x128 MFMA GEMM with split-K partials + fixed-order reduce epilogue (decode batches > 32)."""
    ops.GEMV_VARIANT = ops.TILED
    try:
        k, n = 4096, 768
        e = ops.ext()
        assert e.gemm_ksplit(m, n, k) > 1
        x = torch.randn(m, k)
        w, pg, pc = _mk_linear(n, k)
        y = ops.linear(x.to(DEV), pg, rms_eps=1e-5, out_dtype=torch.float32)
        _close(y, ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)
        yb = ops.linear(x.to(DEV), pg, rms_eps=1e-5)
        _close(yb, ref.linear(x, w, 1e-5, torch.float32), 2e-2, 2e-2)
        xb = x.to(BF16)
        h = torch.randn(m, n)
        hg, mir = h.to(DEV), torch.empty(m, n, dtype=BF16, device=DEV)
        ops.linear_residual(xb.to(DEV), pg, hg, mirror=mir)
        expect = ref.linear_residual(xb, w, h.clone())
        _close(hg, expect, 1e-2, 1e-3)
        torch.testing.assert_close(mir.cpu(), hg.cpu().to(BF16), rtol=0, atol=0)
        gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
        y2 = ops.linear_swiglu(x.to(DEV), PackedLinear.from_dense(gu, DEV), rms_eps=1e-5)
        _close(y2, ref.linear_swiglu(x, gu, 1e-5), 3e-2, 3e-2)
        y_again = ops.linear(x.to(DEV), pg, rms_eps=1e-5, out_dtype=torch.float32)
        assert torch.equal(y, y_again)
    finally:
        ops.GEMV_VARIANT = 0


@pytest.mark.parametrize("m,s", [(48, 1), (128, 1), (256, 1), (96, 2)])
def test_qkv_rope_tiled_splitk(m, s):
    """RoPE + KV-cache write fused into the split-K reduce epilogue."""
    ops.GEMV_VARIANT = ops.TILED
    try:
        h, hkv, dh, k, t = 8, 2, 128, 4096, 80
        b = m // s
        n = (h + 2 * hkv) * dh
        assert ops.ext().gemm_ksplit(m, n, k) > 1
        w = (torch.randn(n, k) * 0.05).to(BF16)
        x = torch.randn(m, k).to(BF16)
        table = ref.rope_table(dh, 256, 500000.0)
        pos = torch.randint(0, 200, (m,), dtype=torch.int32)
        kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
        vc = torch.zeros_like(kc)
        q = ref.linear_qkv_rope(x, w, 1e-5, table, pos, kc, vc, 11, s, h, hkv, dh)
        kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
        pg = PackedLinear.from_dense(w, DEV)
        qg = ops.linear_qkv_rope(x.to(DEV), pg, 1e-5, table.to(DEV), pos.to(DEV), kg, vg,
                                 torch.tensor([11], dtype=torch.int32, device=DEV), s, h, hkv, dh)
        _close(qg, q, 2e-2, 2e-2)
        _close(kg, kc, 2e-2, 2e-2)
        _close(vg, vc, 2e-2, 2e-2)
    finally:
        ops.GEMV_VARIANT = 0


@pytest.mark.parametrize("m,s,n_heads", [(512, 512, 8), (256, 1, 32), (300, 3, 8)])
def test_qkv_rope_direct_epilogue(m, s, n_heads):
    """qkv projection without a K split: the RoPE / KV-cache write runs in the GEMM's own (LDS-staged) epilogue
    (gemm2 FA, 256 x 256 tiles, fused norm) -- against the fp32 oracle, the plain GEMM + RoPE-kernel path, and
    bit for bit across repeated calls; row counts that are not a multiple of the tile included."""
    e = ops.ext()
    hkv, dh, k, t = 8, 128, 4096, 600
    h = n_heads
    b = m // s
    n = (h + 2 * hkv) * dh
    assert e.gemm_qkv_direct_ok(m, 1, k)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    x = torch.randn(m, k).to(BF16)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.randint(0, 1000, (m,), dtype=torch.int32)
    kc = torch.zeros(b, hkv, t, dh, dtype=BF16)
    vc = torch.zeros_like(kc)
    q = ref.linear_qkv_rope(x.float(), w, 1e-5, table, pos, kc, vc, 11, s, h, hkv, dh)
    pg = PackedLinear.from_dense(w, DEV)
    args = (table.to(DEV), pos.to(DEV))
    outs = []
    for _ in range(2):
        kg, vg = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
        qg = torch.empty(m, h, dh, dtype=BF16, device=DEV)
        e.gemm_qkv(x.to(DEV), pg.weight, n, k, args[0], args[1], kg, vg, torch.tensor([11], dtype=torch.int32,
                   device=DEV), s, h, hkv, dh, qg, 1, None, 1e-5, 1)
        outs.append((qg.cpu(), kg.cpu(), vg.cpu()))
    qg, kg, vg = outs[0]
    _close(qg, q, 2e-2, 2e-2)
    _close(kg, kc, 2e-2, 2e-2)
    _close(vg, vc, 2e-2, 2e-2)
    assert all(torch.equal(a, c) for a, c in zip(outs[0], outs[1]))
    # the un-fused path (bf16 qkv store + rope_kv_kernel) agrees to bf16 rounding of the pre-RoPE values
    saved = ops.QKV_DIRECT
    ops.QKV_DIRECT = False
    try:
        kg2, vg2 = torch.zeros_like(kc, device=DEV), torch.zeros_like(vc, device=DEV)
        qg2 = ops.linear_qkv_rope(x.to(DEV), pg, 1e-5, args[0], args[1], kg2, vg2,
                                  torch.tensor([11], dtype=torch.int32, device=DEV), s, h, hkv, dh)
    finally:
        ops.QKV_DIRECT = saved
    _close(qg2.cpu(), qg, 2e-2, 2e-2)
    _close(kg2.cpu(), kg, 2e-2, 2e-2)


def test_rms_scale_bf16_input():
    x = (torch.randn(70, 4096) * 3).to(BF16)
    out = ops.rms_scale(x.to(DEV), 1e-5)
    _close(out, ref.rms_scale(x.float(), 1e-5), 1e-2, 1e-2)


@pytest.mark.parametrize("b,v,k", [(1, 128256, 50), (16, 128256, 50), (3, 32000, 64), (5, 5000, 7), (2, 300, 64)])
def test_topk_candidates_exact(b, v, k):
    logits = torch.randn(b, v) * 4
    logits[0, 17] = logits[0, 99] = logits[0].max() + 1  # ties: lower index first
    if v > 4096:
        logits[-1, 4000:4200] = float("-inf")
    gv, gi = ops.topk_candidates(logits.to(DEV), k)
    rv, ri = ref.topk_sorted(logits, k)
    assert torch.equal(gi.cpu(), ri)
    assert torch.equal(gv.cpu(), rv)


@pytest.mark.parametrize("case", ["block", "flat", "ties"])
def test_topk_candidates_prefilter_fallbacks(case):
    """Chunks whose survivors of the per-thread-maximum prefilter exceed one per thread (a run of 300 large
    logits in one chunk, all-equal logits) take the full select; many exact ties at the threshold keep the
    lowest indices."""
    b, v, k = 3, 128256, 50
    logits = torch.randn(b, v) * 4
    if case == "block":
        logits[:, 8192:8492] = 50.0 + torch.randn(b, 300)
    elif case == "flat":
        logits[:] = 0.0
    else:
        logits[:, ::97] = 30.0  # ~1300 exact ties above everything else, spread over every chunk
    gv, gi = ops.topk_candidates(logits.to(DEV), k)
    rv, ri = ref.topk_sorted(logits, k)
    assert torch.equal(gi.cpu(), ri)
    assert torch.equal(gv.cpu(), rv)


@pytest.mark.parametrize("b,v,k,temp,top_p", [(16, 128256, 50, 1.0, 1.0), (8, 32000, 50, 0.7, 0.9),
                                              (4, 1000, 64, 1.3, 0.5), (2, 50, 1, 1.0, 1.0)])
def test_topk_sample_matches_reference(b, v, k, temp, top_p):
    logits = torch.randn(b, v) * 2
    for step in (5, 6):
        st = torch.tensor([step], dtype=torch.int32, device=DEV)
        got = ops.topk_sample(logits.to(DEV), k, temp, top_p, 1234, st)
        want = ref.topk_sample(logits, k, temp, top_p, 1234, step)
        assert torch.equal(got.cpu(), want)


def test_topk_sample_graph_capturable():
    logits = (torch.randn(4, 128256) * 2).to(DEV)
    st = torch.tensor([9], dtype=torch.int32, device=DEV)
    ops.topk_sample(logits, 50, 0.8, 0.95, 3, st)  # warm workspaces
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = ops.topk_sample(logits, 50, 0.8, 0.95, 3, st)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref.topk_sample(logits.cpu(), 50, 0.8, 0.95, 3, 9))


@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("ks", [1, 3])
@pytest.mark.parametrize("m", [200, 512])
def test_gemm_tile_configs(tile, ks, m):
    """Every gemm2 tile configuration (256x256 / 128x256 / 128x128) x split-K x epilogue, with and
    without the fused RMSNorm statistic, against the fp32 reference."""
    e = ops.ext()
    k, n = 1024, 768
    x = torch.randn(m, k).to(BF16)
    w, pg, _ = _mk_linear(n, k)
    ws = torch.empty(ks * m * (n + 1), dtype=torch.float32, device=DEV)
    wsa = ws if ks > 1 else None
    xg = x.to(DEV)
    for eps in (-1.0, 1e-5):
        r = None if eps < 0 else eps
        out = torch.empty(m, n, dtype=torch.float32, device=DEV)
        e.gemm(xg, pg.weight, n, k, out, ops.MODE_STORE, True, None, ks, wsa, eps, tile)
        _close(out, ref.linear(x, w, r, torch.float32), 1e-2, 2e-3)
        gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
        gp = PackedLinear.from_dense(gu, DEV)
        o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
        e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, wsa, eps, tile)
        _close(o2, ref.linear_swiglu(x, gu, r), 3e-2, 3e-2)
    h = torch.randn(m, n)
    hg, mir = h.to(DEV), torch.empty(m, n, dtype=BF16, device=DEV)
    e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, wsa, -1.0, tile)
    _close(hg, ref.linear_residual(x, w, h.clone()), 1e-2, 1e-3)
    torch.testing.assert_close(mir.cpu(), hg.cpu().to(BF16), rtol=0, atol=0)


@pytest.mark.parametrize("m,k,ks", [(300, 1024, 1), (512, 1056, 1), (256, 992, 3), (700, 4096, 2)])
def test_gemm_full_line_x(m, k, ks):
    """gemm2 (tile 1) with x staged in full 128-B lines (K-tile pairs, swizzled LDS image): every epilogue, with and
    without the fused RMSNorm, including an odd K-tile count (half-used last pair) and split-K ranges that start and
    end mid-pair, against the fp32 reference and reproducible bit for bit. (Its bit-identity with the removed
    fragment-shaped-x pipeline was checked while both existed; gemm4 == gemm2: tests/test_gemm4_gpu.py.)"""
    e = ops.ext()
    n = 768
    x = torch.randn(m, k).to(BF16)
    w, pg, _ = _mk_linear(n, k)
    xg = x.to(DEV)
    ws = torch.empty(ks * m * (n + 1), dtype=torch.float32, device=DEV) if ks > 1 else None
    gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
    gp = PackedLinear.from_dense(gu, DEV)
    h0 = torch.randn(m, n).to(DEV)

    def run():
        outs = []
        for eps in (-1.0, 1e-5):
            o = torch.empty(m, n, dtype=torch.float32, device=DEV)
            e.gemm(xg, pg.weight, n, k, o, ops.MODE_STORE, True, None, ks, ws, eps, 1)
            o2 = torch.empty(m, n // 2, dtype=BF16, device=DEV)
            e.gemm(xg, gp.weight, n, k, o2, ops.MODE_SWIGLU, True, None, ks, ws, eps, 1)
            outs += [o, o2]
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(xg, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws, -1.0, 1)
        return outs + [hg, mir]

    got, again = run(), run()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, again)):
        assert torch.equal(a, b), f"output {i} not reproducible"
    _close(got[0], ref.linear(x, w, None, torch.float32), 1e-2, 2e-3)
    _close(got[2], ref.linear(x, w, 1e-5, torch.float32), 1e-2, 2e-3)


@pytest.mark.parametrize("m,n,k", [(256, 1008, 512), (300, 4096, 1024), (700, 2560, 992)])
def test_gemm_argmax_fused(m, n, k):
    """Greedy lm_head with the argmax in the GEMM epilogue (gemm_argmax) returns exactly what the stored
    fp32 logits + argmax_kernel return (index AND value, with and without the fused RMSNorm), including
    a partial last column tile (n % 256 != 0), a partial row tile, and planted exact ties (first index
    wins, across lanes, waves and workgroups)."""
    e = ops.ext()
    x = torch.randn(m, k).to(BF16)
    w, pg, _ = _mk_linear(n, k)
    # ties: 4 scaled-up rows of W, each repeated at another column (same logits bit for bit), so most
    # row maxima are exact ties -- within a lane group (17/18), across waves (63/64) and workgroups
    wt = w.clone()
    for src, dst in ((3, 700 % n), (17, 18), (n - 300, n - 1), (64, 63)):
        wt[src] = (w[src].float() * 8).to(BF16)
        wt[dst] = wt[src]
    pg = PackedLinear.from_dense(wt, DEV)
    xg = x.to(DEV)
    # the gemm2 plan on both sides (tile 1 here; gemm_argmax off gemm4, whose pairing test_gemm4_gpu checks)
    e.gemm_set_g4_default(0)
    try:
        for eps in (-1.0, 1e-5):
            logits = torch.empty(m, n, dtype=torch.float32, device=DEV)
            e.gemm(xg, pg.weight, n, k, logits, ops.MODE_STORE, True, None, 1, None, eps, 1)
            i0 = torch.empty(m, dtype=torch.int32, device=DEV)
            v0 = torch.empty(m, dtype=torch.float32, device=DEV)
            e.argmax(logits, i0, v0)
            ws = torch.empty(e.gemm_argmax_workspace(m, n), dtype=torch.float32, device=DEV)
            i1 = torch.empty_like(i0)
            v1 = torch.empty_like(v0)
            e.gemm_argmax(xg, pg.weight, n, k, ws, eps, i1, v1)
            torch.cuda.synchronize()
            assert torch.equal(i0.cpu(), i1.cpu()), (eps, (i0 != i1).nonzero()[:8])
            assert torch.equal(v0.cpu(), v1.cpu())
            r = ref.linear(x, wt, None if eps < 0 else eps, torch.float32)
            agree = (r.argmax(-1).to(torch.int32) == i1.cpu()).float().mean().item()
            assert agree > 0.97, agree  # bf16 rounding may flip near-ties against the fp32 reference
        # the op-level API picks the fused path from ARGMAX_FUSED_MIN_M rows on
        idx, val = ops.linear_argmax(xg, pg, 1e-5)
        assert torch.equal(idx.cpu(), i1.cpu()) and torch.equal(val.cpu(), v1.cpu())
    finally:
        e.gemm_set_g4_default(1)


@pytest.mark.parametrize("variant", [12, 15, 18, 21, 22, 26, 7])
@pytest.mark.parametrize("m", [1, 12, 16, 20, 32, 40, 64])
def test_packed_x_variants_and_packed_epilogues(m, variant):
    """Packed-x GEMV variants read the packed copy (ref.pack_act) and match the fp32 reference; the residual /
    SwiGLU epilogues write packed copies of their bf16 outputs that unpack to the row-major outputs exactly.
    Variant 7: the tiled split-K GEMM (decode M > 16), whose reduce epilogue writes the packed copies (it reads
    the row-major x)."""
    if variant == 7 and m <= 16:
        pytest.skip("the tiled GEMM serves decode M > 16")
    k, n = 4096, 768
    rows = ops.packed_rows(m)
    x = torch.randn(m, k).to(BF16)
    w, pg, _ = _mk_linear(n, k)
    xp = ref.pack_act(x, rows).to(DEV)
    ops.GEMV_VARIANT = variant
    try:
        y = torch.empty(m, n, dtype=torch.float32, device=DEV)
        ops._gpu_linear(x.to(DEV), pg, y, ops.MODE_STORE, 1e-5, True, None, xp, None)
        _close(y, ref.linear(x.float(), w, 1e-5, torch.float32), 1e-2, 1e-3)
        h = torch.randn(m, n)
        hg, mir, mp = h.to(DEV), torch.empty(m, n, dtype=BF16, device=DEV), ops.packed_empty(m, n, DEV)
        ops.linear_residual(x.to(DEV), pg, hg, mirror=mir, x_packed=xp, mirror_packed=mp)
        _close(hg, ref.linear_residual(x, w, h.clone()), 1e-2, 1e-3)
        assert torch.equal(mir.cpu(), hg.cpu().to(BF16))
        assert torch.equal(ref.unpack_act(mp.cpu(), m), mir.cpu())
        gu = ref.interleave_gate_up(w[: n // 2], w[n // 2:])
        ap = ops.packed_empty(m, n // 2, DEV)
        y2 = ops.linear_swiglu(x.to(DEV), PackedLinear.from_dense(gu, DEV), rms_eps=1e-5, x_packed=xp, out_packed=ap)
        _close(y2, ref.linear_swiglu(x.float(), gu, 1e-5), 3e-2, 3e-2)
        assert torch.equal(ref.unpack_act(ap.cpu(), m), y2.cpu())
    finally:
        ops.GEMV_VARIANT = 0


@pytest.mark.parametrize("b", [1, 12, 32, 48, 64])
def test_attention_decode_packed_output(b):
    """v5 / v3 (small batch) and the mid-batch v4 stream (33-64 rows) write the packed copy of their output."""
    h, hkv, dh, t = 32, 8, 128, 96
    q = torch.randn(b, 1, h, dh).to(BF16)
    kc = torch.randn(b, hkv, t, dh).to(BF16)
    vc = torch.randn(b, hkv, t, dh).to(BF16)
    kv_start = torch.zeros(b, dtype=torch.int32)
    slot = torch.tensor([t - 1], dtype=torch.int32)
    qg = q.to(DEV)
    assert ops.attention_packs(qg, kc.to(DEV))
    op = ops.packed_empty(b, h * dh, DEV)
    out = ops.attention(qg, kc.to(DEV), vc.to(DEV), slot.to(DEV), kv_start.to(DEV), None, out_packed=op)
    assert torch.equal(ref.unpack_act(op.cpu(), b), out.cpu())


@pytest.mark.parametrize("m,n,k", [(1, 512, 256), (5, 1000, 4096), (130, 257, 96), (256, 128256, 128)])
def test_gemm_f32_exact_mfma(m, n, k):
    """precision='highest' lm_head kernel (gemm_f32.hip, v_mfma_f32_32x32x2_f32) against an fp64 reference: an fp32
    fmaf chain, so the error is a few ulps of sum |a b|; ragged M / N / K exercise the tile guards."""
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV, generator=g)
    w = torch.randn(n, k, device=DEV, generator=g)
    got = ops.linear_f32(x, w)
    want = x.double() @ w.double().t()
    scale = (x.double().abs() @ w.double().abs().t())
    assert float(((got.double() - want).abs() / scale).max()) < 5e-6


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_residual_add_kernel(dt):
    """TP prefill residual epilogue (norm_embed.hip residual_add): h += p; mirror = bf16(h), exact."""
    g = torch.Generator(device=DEV).manual_seed(3)
    h = torch.randn(37, 4096, device=DEV, generator=g)
    p = torch.randn(37, 4096, device=DEV, generator=g).to(dt)
    want = h + p.float()
    mirror = torch.empty(37, 4096, dtype=BF16, device=DEV)
    ops.residual_add_(h, p, mirror)
    assert torch.equal(h, want)
    assert torch.equal(mirror, want.to(BF16))


@pytest.mark.parametrize("kernel", ["v3", "v5"])
@pytest.mark.parametrize("rep", [1, 4, 8, 16])
@pytest.mark.parametrize("t,slot", [(40, 17), (384, 200), (1030, 1029)])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_decode_small_batch_kernels(kernel, rep, t, slot, masked):
    """The two small-batch decode kernels against the fp32 reference: v3 (one workgroup per (row, kv head)) and v5
    (keys split over workgroups, last-arriver merge): left padding that starts inside a split, a row with no valid
    key (zeros), the general key mask, rep up to 16; the packed output copy equals the row-major one."""
    if kernel == "v3" and rep == 16:
        pytest.skip("v3 serves rep <= 8")
    e = ops.ext()
    b, hkv, dh = 3, 2, 128
    h = hkv * rep
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, h, dh).to(BF16)
    kv_start = torch.tensor([0, 37, slot + 1], dtype=torch.int32)
    mask = None
    if masked:
        mask = (torch.rand(b, t) > 0.3).to(torch.uint8)
        mask[:, slot] = 1
        kv_start[1] = 0
    expect = ref.attention(q, kc, vc, slot, kv_start, mask).reshape(b, h * dh)
    try:
        e.attn_set_v5_max_pairs(4096 if kernel == "v5" else 0)
        qd = q.to(DEV)
        kd, vd = kc.to(DEV), vc.to(DEV)
        assert ops.attention_packs(qd, kd)
        packed = ops.packed_empty(b, h * dh, DEV)
        got = ops.attention(qd, kd, vd, torch.tensor([slot], dtype=torch.int32, device=DEV), kv_start.to(DEV),
                            None if mask is None else mask.to(DEV), out_packed=packed)
        again = ops.attention(qd, kd, vd, torch.tensor([slot], dtype=torch.int32, device=DEV), kv_start.to(DEV),
                              None if mask is None else mask.to(DEV))
        torch.cuda.synchronize()
    finally:
        e.attn_set_v5_max_pairs(-1)
    _close(got, expect, 2e-2, 2e-2)
    assert torch.equal(got, again)  # tickets reset themselves: a second call merges the same way
    if not masked:
        assert got[2].float().abs().max().item() == 0.0
    assert torch.equal(ref.unpack_act(packed.cpu(), b), got.cpu())


@pytest.mark.parametrize("wpp", [1, 2, 4, 8])
@pytest.mark.parametrize("rep", [1, 4, 8, 16])
@pytest.mark.parametrize("t,slot", [(40, 17), (384, 200), (1030, 1029)])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_decode_mfma_v6(wpp, rep, t, slot, masked):
    """Decode attention on the matrix cores (attn_decode_mma.hip, v6) forced at every waves-per-pair geometry against
    the fp32 reference: left padding that starts inside a 32-key step, a row with no valid key (zeros), the general key
    mask, rep 1..16 (the heads of a pair are the MFMA columns); the packed output copy equals the row-major one and a
    second call is identical (no state between calls)."""
    e = ops.ext()
    b, hkv, dh = 3, 2, 128
    h = hkv * rep
    kc, vc = _cache(b, hkv, t, dh)
    q = torch.randn(b, 1, h, dh).to(BF16)
    kv_start = torch.tensor([0, 37, slot + 1], dtype=torch.int32)
    mask = None
    if masked:
        mask = (torch.rand(b, t) > 0.3).to(torch.uint8)
        mask[:, slot] = 1
        kv_start[1] = 0
    expect = ref.attention(q, kc, vc, slot, kv_start, mask).reshape(b, h * dh)
    try:
        e.attn_set_v6(2)
        e.attn_set_v6_wpp(wpp)
        qd, kd, vd = q.to(DEV), kc.to(DEV), vc.to(DEV)
        sl = torch.tensor([slot], dtype=torch.int32, device=DEV)
        md = None if mask is None else mask.to(DEV)
        assert e.attn_decode_splits(b, hkv, t, rep) == 1 and e.attn_decode_packs(b, hkv, rep)
        packed = ops.packed_empty(b, h * dh, DEV)
        got = ops.attention(qd, kd, vd, sl, kv_start.to(DEV), md, out_packed=packed)
        again = ops.attention(qd, kd, vd, sl, kv_start.to(DEV), md)
        torch.cuda.synchronize()
    finally:
        e.attn_set_v6(0)
        e.attn_set_v6_wpp(0)
    _close(got, expect, 2e-2, 2e-2)
    assert torch.equal(got, again)
    if not masked:
        assert got[2].float().abs().max().item() == 0.0
    assert torch.equal(ref.unpack_act(packed.cpu(), b), got.cpu())


@pytest.mark.parametrize("spl", [1, 2])
@pytest.mark.parametrize("b,hkv,rep", [(1, 1, 8), (2, 8, 4), (4, 2, 1), (1, 2, 16), (3, 1, 8), (24, 1, 8), (32, 1, 8)])
@pytest.mark.parametrize("t,slot", [(40, 17), (200, 199), (384, 300), (512, 130)])
def test_qkv_attention_fused_launch(b, hkv, rep, t, slot, spl):
    """The fused small-batch decode launch (gemv.hip qkv_attn_kernel: qkv GEMV + RoPE + KV write on one set of
    workgroups, the attention on another that prefetches its K / V step and waits for the write-through publish)
    against the fp32 reference of linear_qkv_rope + attention: left padding inside a split, a row with no valid key,
    the new key at the end of a 32-key step or of a 128-key split; the cache rows it wrote equal the unfused kernel's,
    the packed output equals the row-major one, and a second launch agrees (the counters reset themselves); with the
    qkv GEMV's K over one or two workgroups per column group (spl)."""
    e = ops.ext()
    dh, k = 128, 1024
    h = hkv * rep
    n = (h + 2 * hkv) * dh
    torch.manual_seed(b * 100 + t + rep)
    x = torch.randn(b, k).to(BF16)
    w = (torch.randn(n, k) * 0.03).to(BF16)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.full((b,), slot, dtype=torch.int32)
    kc0, vc0 = _cache(b, hkv, t, dh)
    kv_start = (torch.tensor([0, 37, slot + 1] + [5 * i % 60 for i in range(b - 3)][:max(0, b - 3)], dtype=torch.int32)[:b]
                if b > 1 else torch.tensor([3], dtype=torch.int32))
    kcr, vcr = kc0.clone(), vc0.clone()
    q = ref.linear_qkv_rope(x.float(), w, 1e-5, table, pos, kcr, vcr, slot, 1, h, hkv, dh)
    expect = ref.attention(q.reshape(b, 1, h, dh), kcr, vcr, slot, kv_start).reshape(b, h * dh)
    from jax_llama_amd.models.weights import PackedLinear
    pw = PackedLinear.from_dense(w, DEV)
    kd, vd = kc0.to(DEV), vc0.to(DEV)
    xd = x.to(DEV)
    sl = torch.tensor([slot], dtype=torch.int32, device=DEV)
    splits = e.qkv_attn_splits(b, b, hkv, rep, t, n, ops._num_cus(xd.device), spl)
    if spl == 2 and splits == 0:  # (twice the qkv workgroups: this grid no longer fits the CUs at once)
        assert e.qkv_attn_splits(b, b, hkv, rep, t, n, ops._num_cus(xd.device), 1) > 0
        pytest.skip("the split qkv grid does not fit the CUs")
    assert splits == (t + 127) // 128, (splits, e.qkv_attn_occupancy(b, rep, spl))
    packed = ops.packed_empty(b, h * dh, DEV)
    got = ops.linear_qkv_attention(xd, pw, 1e-5, table.to(DEV), pos.to(DEV), kd, vd, sl, kv_start.to(DEV), h, hkv, dh,
                                   splits, out_packed=packed, spl=spl)
    again = ops.linear_qkv_attention(xd, pw, 1e-5, table.to(DEV), pos.to(DEV), kd, vd, sl, kv_start.to(DEV), h, hkv,
                                     dh, splits, spl=spl)
    torch.cuda.synchronize()
    _close(got, expect, 2e-2, 2e-2)
    assert torch.equal(got, again)
    assert torch.equal(ref.unpack_act(packed.cpu(), b), got.cpu())
    if b > 2:
        assert got[2].float().abs().max().item() == 0.0  # kv_start = slot + 1: no valid key
    # the cache rows: as the unfused qkv GEMV of the same geometry (variant 1: one tile x 4 waves; spl 2: variant 16,
    # the same with K over 2 workgroups) writes them
    ku, vu = kc0.to(DEV), vc0.to(DEV)
    try:
        ops.GEMV_VARIANT = 1 if spl == 1 else 16
        ops.linear_qkv_rope(xd, pw, 1e-5, table.to(DEV), pos.to(DEV), ku, vu, sl, 1, h, hkv, dh)
        torch.cuda.synchronize()
    finally:
        ops.GEMV_VARIANT = 0
    if b <= 16:
        assert torch.equal(ku.cpu(), kd.cpu()) and torch.equal(vu.cpu(), vd.cpu())
    else:  # (M > 16: the unfused GEMV cuts K over 8 waves, the fused launch over 4 -- another summation order)
        _close(kd, ku, 1e-2, 1e-2)
        _close(vd, vu, 1e-2, 1e-2)


@pytest.mark.parametrize("tp", [False, True])
@pytest.mark.parametrize("nt", [2, 1])
@pytest.mark.parametrize("b,t,slot,spl", [(1, 40, 17, 2), (1, 384, 300, 1), (3, 200, 199, 2), (16, 512, 130, 2)])
def test_qkv_attention_fused_o_projection(b, t, slot, spl, nt, tp):
    """The fused decode launch with the o projection on its last workgroups (gemv.hip qa_o_proj): the residual after
    the launch equals the standalone GEMV of the same geometry applied to the launch's attention output -- bit for bit
    (variant 6 / 1: 2 / 1 tiles x 4 waves, the same per-wave k-step order and the same epilogue), in the residual
    epilogue (world 1) and the TP granule exchange (a world-1 fused all-reduce instance) -- and the fp32 reference of
    h + attention @ Wo^T within bf16 tolerance; the packed mirror equals the row-major one; a second step agrees."""
    from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
    e = ops.ext()
    dh, k, hkv, rep = 128, 1024, 1, 8
    h_ = hkv * rep
    n, d = (h_ + 2 * hkv) * dh, 2048
    torch.manual_seed(b * 10 + t)
    x = torch.randn(b, k).to(BF16)
    w = (torch.randn(n, k) * 0.03).to(BF16)
    wo = (torch.randn(d, h_ * dh) * 0.03).to(BF16)
    h0 = torch.randn(b, d)
    table = ref.rope_table(dh, 1024, 500000.0)
    pos = torch.full((b,), slot, dtype=torch.int32)
    kc0, vc0 = _cache(b, hkv, t, dh)
    kv_start = torch.tensor([3 * i % 50 for i in range(b)], dtype=torch.int32)
    pw, pwo = PackedLinear.from_dense(w, DEV), PackedLinear.from_dense(wo, DEV)
    xd, sl = x.to(DEV), torch.tensor([slot], dtype=torch.int32, device=DEV)
    car = CustomAllReduce.local(max_bytes=CustomAllReduce.fused_bytes(d)) if tp else None
    e.qkv_attn_set_o_nt(nt)
    try:
        og = e.qkv_attn_o_groups(b, rep, d, h_ * dh)
        assert og == (d // 16 + nt - 1) // nt
        splits = e.qkv_attn_splits(b, b, hkv, rep, t, n, ops._num_cus(xd.device), spl, og)
        if splits == 0:
            pytest.skip("this grid does not fit the CUs at once")

        def step():
            kd, vd = kc0.to(DEV), vc0.to(DEV)
            hd = h0.to(DEV)
            hbd = torch.empty(b, d, dtype=BF16, device=DEV)
            hbp = ops.packed_empty(b, d, DEV)
            a = ops.linear_qkv_attention(xd, pw, 1e-5, table.to(DEV), pos.to(DEV), kd, vd, sl, kv_start.to(DEV), h_,
                                         hkv, dh, splits, spl=spl,
                                         o=(pwo, hd, hbd, hbp, car._live() if tp else 0))
            torch.cuda.synchronize()
            return a, hd, hbd, hbp

        a, hd, hbd, hbp = step()
        a2, hd2, hbd2, _ = step()
        # the standalone GEMV of the same geometry on the launch's own attention output
        hu = h0.to(DEV)
        hbu = torch.empty(b, d, dtype=BF16, device=DEV)
        try:
            ops.GEMV_VARIANT = 6 if nt == 2 else 1
            if tp:
                ops.linear_tp_residual(a, pwo, hu, hbu, car._live())
            else:
                ops.linear_residual(a, pwo, hu, mirror=hbu)
            torch.cuda.synchronize()
        finally:
            ops.GEMV_VARIANT = 0
    finally:
        e.qkv_attn_set_o_nt(2)
        if car is not None:
            car.close()
    assert torch.equal(hd, hu) and torch.equal(hbd, hbu)
    assert torch.equal(hbd, hd.to(BF16))
    assert torch.equal(ref.unpack_act(hbp.cpu(), b), hbd.cpu())
    assert torch.equal(a, a2) and torch.equal(hd, hd2) and torch.equal(hbd, hbd2)
    kcr, vcr = kc0.clone(), vc0.clone()
    q = ref.linear_qkv_rope(x.float(), w, 1e-5, table, pos, kcr, vcr, slot, 1, h_, hkv, dh)
    att = ref.attention(q.reshape(b, 1, h_, dh), kcr, vcr, slot, kv_start).reshape(b, h_ * dh)
    _close(a, att, 2e-2, 2e-2)
    _close(hd, h0 + a.float().cpu() @ wo.float().t(), 1e-2, 1e-2)


@pytest.mark.parametrize("m,n,k,ks,tile", [(96, 1024, 512, 2, 7), (256, 8192, 3584, 4, 7), (200, 2048, 1024, 3, 1),
                                           (130, 4096, 1024, 2, 11), (65, 512, 256, 2, 17)])
def test_tiled_tp_residual_fused_reduce(m, n, k, ks, tile):
    """Row-parallel tiled projection with the TP all-reduce and residual add in its split-K reduce (gemm.hip
    gemm_reduce_tp_kernel, MODE_TPRESID) on a world-1 fused instance: bit-identical h and mirror to the same plan's
    bf16 partial + the standalone residual all-reduce (car_reduce_kernel), over several calls (both parities,
    counters advancing) and interleaved with the GEMV's fused epilogue on the same counters; and h + x @ W^T of the
    fp32 reference within bf16 tolerance. Includes the Llama-3-70B MP 8 down projection at B = 256 and a gemm5 plan."""
    from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
    e = ops.ext()
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    w = PackedLinear.random(n, k, DEV, 0.02, g)
    x = (torch.randn(m, k, device=DEV, generator=g)).to(BF16)
    h0 = torch.randn(m, n, device=DEV, generator=g)
    fused = CustomAllReduce.local(max_bytes=CustomAllReduce.fused_bytes(max(n, 8192)))
    coll = CustomAllReduce.local(max_bytes=16 << 20)
    try:
        assert fused.can_fuse_tiled(m, n)
        g5 = tile in (11, 12)
        wsn = (e.gemm5_ksplit(k, ks) if g5 else ks) * m * (n + 1)
        ws = torch.empty(wsn, dtype=torch.float32, device=DEV)
        hs = torch.randn(16, 512, device=DEV, generator=g)
        xs = torch.randn(16, 512, device=DEV, generator=g).to(BF16)
        ws_small = PackedLinear.random(512, 512, DEV, 0.02, g)
        for rep in range(3):
            h1, h2 = h0.clone(), h0.clone()
            hb1 = torch.empty(m, n, dtype=BF16, device=DEV)
            hb2 = torch.empty_like(hb1)
            e.gemm_tp_residual(fused._live(), x, w.weight, n, k, h1, hb1, ks, ws, tile)
            part = torch.empty(m, n, dtype=BF16, device=DEV)
            e.gemm(x, w.weight, n, k, part, ops.MODE_STORE, True, None, ks, ws, -1.0, tile)
            coll.all_reduce_residual_(part, h2, hb2)
            torch.cuda.synchronize()
            assert torch.equal(h1, h2) and torch.equal(hb1, hb2), rep
            # a GEMV call with the fused epilogue on the same instance (shared per-workgroup counters)
            hsb = torch.empty(16, 512, dtype=BF16, device=DEV)
            ops.linear_tp_residual(xs, ws_small, hs, hsb, fused._live())
        torch.cuda.synchronize()
        assert fused.error() == 0 and coll.error() == 0
    finally:
        fused.close()
        coll.close()
    want = h0.cpu() + x.float().cpu() @ w.dense().float().cpu().t()
    _close(h1, want, 2e-2, 2e-2)
