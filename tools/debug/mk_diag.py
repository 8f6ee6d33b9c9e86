import sys, os, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from jax_llama_amd import ops
from jax_llama_amd.config import get_preset
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.models.llama import mask_to_kv_start
from helpers import rel_err

DEV = "cuda"

def run(model, toks, mk):
    ops.DECODE_MK = mk
    b, s = toks.shape
    cache = model.init_cache(b, s + 8)
    kv_start = torch.zeros(b, dtype=torch.int32, device=DEV)
    pos = torch.arange(s, dtype=torch.int32, device=DEV).repeat(b, 1)
    logits, _, _, _ = model.forward_tokens(toks.to(DEV), pos.reshape(-1), cache, 0, kv_start, None, logits_mode="last")
    cache.advance(s)
    nxt = logits.float().argmax(-1).to(torch.int32)
    pos1 = torch.full((b,), s, dtype=torch.int32, device=DEV)
    l1, h1, _, _ = model.forward_tokens(nxt[:, None], pos1, cache, cache.index_t, kv_start, None, logits_mode="last")
    torch.cuda.synchronize()
    L = model.config.num_hidden_layers
    return dict(h=h1.float().cpu(), k=[cache.k[l, :, :, s].float().cpu() for l in range(L)],
                v=[cache.v[l, :, :, s].float().cpu() for l in range(L)])

for dims in [dict(), dict(intermediate_size=4096)]:
  for layers in (1, 2):
    cfg = get_preset("llama3-8b", num_hidden_layers=layers, max_seq_len=512, **dims)
    model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).init_random(seed=3)
    for s in (9, 40, 70, 200):
        g = torch.Generator().manual_seed(5)
        toks = torch.randint(0, cfg.vocab_size, (1, s), generator=g, dtype=torch.int32)
        a = run(model, toks, True)
        err = ops.decode_mk_error(DEV)
        b = run(model, toks, False)
        print(json.dumps({"layers": layers, "dims": dims, "prompt": s, "mk_err": err, "h": rel_err(a["h"], b["h"]),
                          "k": [rel_err(x, y) for x, y in zip(a["k"], b["k"])],
                          "v": [rel_err(x, y) for x, y in zip(a["v"], b["v"])]}), flush=True)
