"""Diagnostic: whole-model logits (GPU vs CPU path) with the decode GEMM variant pinned, per variant.
Run from the repo root on a GPU box: python tools/debug/variant_sweep_model.py"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from jax_llama_amd import ops  # noqa: E402
from jax_llama_amd.models import LLaMAForCausalLM  # noqa: E402
from helpers import build, gpu_config, rel_err  # noqa: E402

for kv in (2, 1):
    cfg = gpu_config(num_attention_heads=2, num_key_value_heads=kv)
    model_cpu, oracle, sd, params = build(cfg, seed=0)
    gpu = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).load_params(params)
    for m_rows in (1, 5, 20):
        toks = torch.randint(0, cfg.vocab_size, (3, m_rows), dtype=torch.int32)
        lc = model_cpu(toks).logits
        for v in (0, 1, 4, 5, 6, 7, 9, 10, 11):
            ops.GEMV_VARIANT = v
            try:
                lg = gpu(toks).logits.cpu()
                print(f"kv={kv} M={3 * m_rows} variant={v} rel_err={rel_err(lg, lc):.4f}", flush=True)
            except Exception as ex:  # noqa: BLE001
                print(f"kv={kv} M={3 * m_rows} variant={v} error {ex}", flush=True)
        ops.GEMV_VARIANT = 0
