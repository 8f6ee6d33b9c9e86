"""Debug: reproducibility of the split-K skinny GEMM (variant 4)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from jax_llama_amd import ops
from jax_llama_amd.models.weights import PackedLinear
from jax_llama_amd.ops import reference as ref

ops.GEMV_VARIANT = 4
torch.manual_seed(0)
for (m, n, k) in [(9, 768, 4096), (1, 768, 4096), (16, 4096, 4096), (64, 768, 4096)]:
    x = torch.randn(m, k, device="cuda")
    w = PackedLinear.from_dense((torch.randn(n, k) * 0.05).to(torch.bfloat16), "cuda")
    w2 = PackedLinear.from_dense((torch.randn(n, k) * 0.05).to(torch.bfloat16), "cuda")
    base = ops.linear(x, w, rms_eps=1e-5, out_dtype=torch.float32)
    exp = ref.linear(x.cpu(), w.dense().cpu(), 1e-5, torch.float32)
    nbad = 0
    for it in range(30):
        _ = ops.linear(x, w2, rms_eps=1e-5, out_dtype=torch.float32)   # other data through the same slabs
        y = ops.linear(x, w, rms_eps=1e-5, out_dtype=torch.float32)
        if not torch.equal(y, base):
            d = (y - base).abs()
            nbad += 1
            if nbad <= 3:
                idx = (d > 0).nonzero()
                print(f"m={m} it={it}: {int((d>0).sum())} elems differ, max {d.max().item():.3e}, first {idx[:4].tolist()}")
    err = (base.cpu() - exp).abs().max().item()
    print(f"m={m} n={n} k={k}: {nbad}/30 runs differ; err vs ref {err:.3e}", flush=True)
