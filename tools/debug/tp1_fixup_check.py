"""Debug: TP1 reference of the TP test model (70B dims, 2 layers) with the split-K fixup on/off and attention
v4 on/off: compare greedy sequences and prefill logits."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from helpers import left_padded_batch
from jax_llama_amd import ops
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.engine import GenerationConfig
from test_tp_gpu import _config, _gpu_params

e = ops.ext()
print("SKINNY_MAX_M", e.SKINNY_MAX_M)
cfg = _config("70b")
params = _gpu_params(cfg, seed=21)
toks, mask = left_padded_batch([5, 9, 12, 12], 12, cfg.vocab_size, pad=2, seed=4)
pos = mask.cumsum(-1) - 1
gc = GenerationConfig(max_length=12 + 16, do_sample=False, pad_token_id=2, eos_token_id=-1)
res = {}
for fix in (True, False):
    for attn in (2, 5):
        e.gemm_set_fixup(fix)
        e.attn_set_impl(attn, 2048)
        ref = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).load_params(params)
        lr = ref(toks, attention_mask=mask, position_ids=pos).logits.float().cpu()
        sr = ref.generate(toks, attention_mask=mask, generation_config=gc).sequences.cpu()
        res[(fix, attn)] = (lr, sr)
        del ref
        torch.cuda.empty_cache()
base = res[(False, 5)]
for k, (lr, sr) in res.items():
    print(k, "logits max|diff|", float((lr - base[0]).abs().max()), "seq equal", torch.equal(sr, base[1]))
    if not torch.equal(sr, base[1]):
        print("  diff positions", (sr != base[1]).nonzero().tolist()[:10])
