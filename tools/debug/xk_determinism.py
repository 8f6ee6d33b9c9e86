import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from jax_llama_amd import ops
from jax_llama_amd.models.weights import PackedLinear
BF16 = torch.bfloat16
DEV = "cuda"
e = ops.ext()
for (m, n, k, ks) in [(2048, 4096, 4096, 2), (512, 1024, 1024, 2), (256, 8192, 1024, 4)]:
    torch.manual_seed(0)
    x = torch.randn(m, k).to(BF16).to(DEV)
    w = (torch.randn(n, k) * 0.05).to(BF16)
    pg = PackedLinear.from_dense(w, DEV)
    h0 = torch.randn(m, n, device=DEV)
    floats, counts = e.gemm4_xk_workspace(m, n, ks)
    ws = torch.zeros(floats, device=DEV)
    cnt = torch.zeros(counts, dtype=torch.int32, device=DEV)
    slabs = torch.empty(ks * m * (n + 1), device=DEV)
    def run(tile):
        hg, mir = h0.clone(), torch.empty(m, n, dtype=BF16, device=DEV)
        e.gemm(x, pg.weight, n, k, hg, ops.MODE_RESIDUAL, True, mir, ks, ws if tile == 8 else slabs, -1.0, tile,
               cnt if tile == 8 else None)
        torch.cuda.synchronize()
        return hg
    red = run(7)
    for r in range(4):
        a = run(8)
        d = (a - red).abs()
        bad = (d > 1e-4).nonzero()
        print(m, n, k, ks, "run", r, "maxdiff", d.max().item(), "nbad", bad.shape[0], "cnt", cnt.abs().sum().item(), flush=True)
        if bad.shape[0]:
            rows = torch.unique(bad[:, 0] // 128).tolist()[:20]
            cols = torch.unique(bad[:, 1] // 128).tolist()[:20]
            print("  row blocks", rows, "col blocks", cols, "first", bad[:4].tolist(), flush=True)
