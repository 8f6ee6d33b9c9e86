"""Localise a decode-attention mismatch: impl 1 vs 2 on structured inputs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from jax_llama_amd import ops
from jax_llama_amd.ops import reference as ref
e = ops.ext()
B, HKV, T, DH = 3, 2, 40, 128
for rep in (1, 4):
    H = HKV * rep
    for name in ("ones_v", "zero_k", "random"):
        torch.manual_seed(0)
        kc = (torch.randn(B, HKV, T, DH) * 0.5).bfloat16()
        vc = torch.randn(B, HKV, T, DH).bfloat16()
        q = torch.randn(B, 1, H, DH).bfloat16()
        if name == "ones_v":
            vc = torch.ones_like(vc)
        if name == "zero_k":
            kc = torch.zeros_like(kc)
            vc = torch.arange(T).float().view(1, 1, T, 1).expand(B, HKV, T, DH).bfloat16().contiguous()
        slot = 17
        ks = torch.tensor([0, 5, 0], dtype=torch.int32)
        exp = ref.attention(q, kc, vc, slot, ks).reshape(B, H * DH)
        for impl in (1, 2):
            e.attn_set_impl(impl, 4096)
            got = ops.attention(q.cuda(), kc.cuda(), vc.cuda(), torch.tensor([slot], dtype=torch.int32, device="cuda"),
                                ks.cuda()).float().cpu()
            err = (got - exp).abs().max().item()
            print(rep, name, impl, "err", round(err, 4), "got[0,:4]", got[0, :4].tolist(), "exp", exp[0, :4].tolist(),
                  "got[1,128:132]", got[1, 128:132].tolist(), flush=True)
