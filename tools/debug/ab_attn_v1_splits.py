"""A/B of decode attention geometry at small batch (graph-replayed, 20 calls per replay)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402

e = ops.ext()


def run(b, label):
    kc = torch.randn(b, 8, 384, 128, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(b, 1, 32, 128, device="cuda").to(torch.bfloat16)
    slot = torch.tensor([160], dtype=torch.int32, device="cuda")
    ks = torch.zeros(b, dtype=torch.int32, device="cuda")
    for _ in range(3):
        ops.attention(q, kc, vc, slot, ks)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            ops.attention(q, kc, vc, slot, ks)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"b": b, "cfg": label, "nsplit": e.attn_decode_splits(b, 8, 384, 4),
                      "us": round(e0.elapsed_time(e1) * 1000 / 20, 2)}), flush=True)


for b in (1, 8, 32, 64, 128, 256):
    e.attn_set_impl(2, 2048)
    e.attn_set_v3_max_pairs(1 << 30)
    run(b, "v3")
    e.attn_set_v3_max_pairs(0)
    run(b, "v1")
    for tgt in (8, 32, 128, 512, 2048):
        e.attn_set_impl(2, tgt)
        e.attn_set_impl(2, -1)  # v2 at any batch, keep the waves target
        run(b, f"v2_target{tgt}")
    e.attn_set_impl(2, 2048)
    e.attn_set_impl(2, 2048)
    e.attn_set_v3_max_pairs(1024)
