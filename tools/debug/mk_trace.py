import sys, os, json
sys.path.insert(0, os.getcwd())
import torch
from jax_llama_amd import ops
from jax_llama_amd.config import get_preset
from jax_llama_amd.models import LLaMAForCausalLM
from jax_llama_amd.runtime.benchmark import decode_latency

DEV = "cuda"
cfg = get_preset("llama3-8b", max_seq_len=2048)
model = LLaMAForCausalLM(cfg, device=DEV, _do_init=False).init_random(seed=1)
ops.DECODE_MK = True
e = ops.ext()
tr = torch.zeros(e.decode_mk_trace_words(), dtype=torch.int64, device=DEV)
for late in (0, 1):
    ops.DECODE_MK_PREFETCH_LATE = late
    p = decode_latency(model, 1, 128, 256, seed=7)
    print(json.dumps({"decode_ms": p["decode_ms_per_token"], "prefetch_late": late}))
ops.DECODE_MK_TRACE = tr
ops.DECODE_MK_PREFETCH_LATE = int(os.environ.get("MK_LATE", "0"))
# one eager step with tracing
from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
from jax_llama_amd.runtime.benchmark import synthetic_prompts
eng = DecodeEngine(model, 1, 384, use_graph=False)
eng.gc = GenerationConfig(max_length=384, do_sample=False, pad_token_id=0, eos_token_id=-1)
eng.prefill(synthetic_prompts(cfg.vocab_size, 1, 128, 7), None)
eng._decode_step()
torch.cuda.synchronize()
G = tr.numel() // 50
t = tr.view(10, 5, G).cpu().double() / 100.0  # us (100 MHz), per wave
t[t <= 0] = float("nan")
t0 = t[0, 0].nan_to_num(1e30).min()
def q(x, f):
    x = x[~torch.isnan(x)]
    return round(float(f(x)), 2) if x.numel() else None
names = ["qkv", "attn", "wo", "w13", "w2"]
for ph in range(10):
    ev = t[ph] - t0
    wait = (ev[1] - ev[0]); stage = (ev[2] - ev[1]); stream = (ev[3] - ev[2]); epi = (ev[4] - ev[3])
    row = {"phase": f"L{ph // 5}.{names[ph % 5]}", "entry_med": q(ev[0], torch.median),
           "release_min": q(ev[1], torch.min), "release_max": q(ev[1], torch.max),
           "last_entry": q(ev[0], torch.max), "done_med": q(ev[4], torch.median), "done_max": q(ev[4], torch.max)}
    if ph % 5 != 1:
        row.update({"stage_med": q(stage, torch.median), "stream_med": q(stream, torch.median),
                    "stream_max": q(stream, torch.max), "epi_med": q(epi, torch.median), "epi_max": q(epi, torch.max),
                    "epi_p99": q(epi, lambda x: x.quantile(0.99)), "streamdone_max": q(ev[3], torch.max)})
    print(json.dumps(row))
