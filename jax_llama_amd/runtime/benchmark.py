"""Measurement helpers shared by ``bench.py`` and ``tools/``: decode latency points (hipGraph-replayed
decode steps timed with HIP events, prefill excluded) and end-to-end generate throughput.

BASELINE.md's protocol: decode tokens/s = B x generated tokens / decode wall time, hipGraph replay,
prefill excluded; prompts of 128 synthetic tokens, max_gen_len 256, B in {1, 8, 32}, greedy.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .engine import DecodeEngine, GenerationConfig


def synthetic_prompts(vocab: int, batch: int, prompt_len: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(3, vocab, (batch, prompt_len), generator=g, dtype=torch.int32)


def decode_latency(model, batch: int, prompt_len: int = 128, gen_len: int = 256, steps: Optional[int] = None,
                   seed: int = 0, barrier=None, do_sample: bool = False) -> Dict[str, float]:
    """Prefill ``batch`` prompts into a ``prompt_len + gen_len`` cache (``prefill_ms``: the second, warm prefill; the
    first autotunes), capture the decode step (every layer, lm_head, sampler, state update), prefill again, then time
    ``steps`` replays of it -- by default every step of a ``gen_len``-token generation (``gen_len - 1`` replays after
    the prefill's first token, cache length from ``prompt_len + 1`` up), so attention is weighted as in a real
    generation (``kv_len_mean`` reports the mean cache length the steps covered; reference generation.py:35:
    max_length = S + max_gen_len). Every rank of a TP group must call this with the same arguments."""
    steps = gen_len - 1 if steps is None else steps
    assert 1 <= steps <= gen_len - 1, "replays must stay inside the cache"
    max_len = prompt_len + gen_len
    eng = DecodeEngine(model, batch, max_len, use_graph=True)
    gc = GenerationConfig(max_length=max_len, do_sample=do_sample, temperature=0.8, top_p=0.95, top_k=50,
                          pad_token_id=0, eos_token_id=-1)
    eng.gc = gc
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    eng.prefill(prompts, None)  # cold: autotunes new prefill shapes and grows the workspaces; not timed
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    eng.prefill(prompts, None)  # warm prefill: ``prefill_ms``
    ev1.record()
    eng._decode_step()  # eager step: sizes the workspaces before capture
    eng.keep_graph = True
    eng._ensure_graph()
    eng._graph.replay()
    torch.cuda.synchronize(dev)
    ttft_ms = ev0.elapsed_time(ev1)
    kernels = graph_kernels(eng._graph)
    eng.prefill(prompts, None)  # back to the first decode position: the timed replays cover the whole window
    torch.cuda.synchronize(dev)
    if barrier is not None:
        barrier()
    ev0.record()
    for _ in range(steps):
        eng._graph.replay()
    ev1.record()
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / steps
    model.comm.check()
    del eng
    return {"batch": batch, "decode_ms_per_token": round(ms, 4),
            "decode_tokens_per_sec": round(batch * 1000.0 / ms, 2), "prefill_ms": round(ttft_ms, 3),
            "steps": steps, "kv_len_mean": round(prompt_len + 1 + (steps - 1) / 2, 1),
            # launches of one decode step, counted from the captured graph's kernel nodes (every layer, lm_head,
            # sampler, state update)
            "kernels_per_step": kernels,
            "kernels_per_layer": round(kernels / model.config.num_hidden_layers, 2) if kernels >= 0 else None}


def graph_kernels(graph) -> int:
    """Kernel nodes of a captured torch.cuda.CUDAGraph (hipGraphGetNodes; -1 when the raw graph is unavailable)."""
    from .. import ops
    try:
        return int(ops.ext().graph_kernel_nodes(int(graph.raw_cuda_graph())))
    except (AttributeError, RuntimeError):
        return -1


def time_to_first_token(model, batch: int, prompt_len: int, reps: int = 3, seed: int = 0,
                        barrier=None) -> Dict[str, float]:
    """Prefill of ``batch`` synthetic prompts of ``prompt_len`` tokens up to the first generated token
    (every layer's GEMMs + flash attention + KV-cache writes, last-position lm_head, greedy argmax),
    timed with HIP events after one warm-up prefill (autotune, workspace growth). Median of ``reps``."""
    eng = DecodeEngine(model, batch, prompt_len + 8, use_graph=False)
    gc = GenerationConfig(max_length=prompt_len + 8, do_sample=False, pad_token_id=0, eos_token_id=-1)
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    eng.prefill_only(prompts, None, gc)
    torch.cuda.synchronize(dev)
    if barrier is not None:
        barrier()
    times = []
    for _ in range(reps):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        eng.prefill_only(prompts, None, gc)
        ev1.record()
        torch.cuda.synchronize(dev)
        times.append(ev0.elapsed_time(ev1))
    model.comm.check()
    del eng
    ms = sorted(times)[len(times) // 2]
    return {"batch": batch, "prompt_len": prompt_len, "ttft_ms": round(ms, 3),
            "prefill_tokens_per_sec": round(batch * prompt_len * 1000.0 / ms, 1)}


def generate_tokens_per_sec(model, batch: int, prompt_len: int, gen_len: int, gc: GenerationConfig,
                            seed: int = 0, reps: int = 1, barrier=None) -> Dict[str, float]:
    """Whole ``generate`` calls (prefill + every decode step + sampler), output tokens per second."""
    import time
    prompts = synthetic_prompts(model.config.vocab_size, batch, prompt_len, seed)
    dev = model.device
    model.generate(prompts, generation_config=gc)  # warm-up: engine, capture, autotune
    torch.cuda.synchronize(dev)
    if barrier is not None:
        barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        model.generate(prompts, generation_config=gc)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"batch": batch, "ms_per_generate": round(1000 * dt, 2), "tokens_per_sec": round(batch * gen_len / dt, 2)}


def _sclk_levels():
    """(current level line, max level line) of the shader clock from sysfs (pp_dpm_sclk), or (None, None)."""
    import glob
    try:
        for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk")):
            lines = [ln.strip() for ln in open(f) if ln.strip()]
            if lines:
                cur = next((ln for ln in lines if ln.endswith("*")), None)
                return cur, lines[-1]
    except OSError:
        pass
    return None, None


def calibration(device) -> Dict[str, object]:
    """Fixed-work probes that tell a slower box from a kernel regression (bench.py ``calibration``):
      * bf16 GEMM TFLOP/s of one fixed 8192^3 shape on this framework's tiled GEMM and on the vendor library
        (torch.mm -> hipBLASLt);
      * ``stream_read_tbps``: a 2 GiB read-only stream through the repo's grid-strided streaming-read kernel
        (norm_embed.hip prefetch_kernel, 16 loads in flight per lane, 4 workgroups per CU); ``stream_read_seq_tbps``:
        the same bytes in the decode kernels' pattern (one contiguous range per wave, stream_probe_kernel) -- the box's
        read roofline, which bench.py divides the streamed bytes by (``hbm_roofline_ms_per_token_box``) beside the fixed
        6.29 TB/s of the guide's copy measurement; ``copy_tbps`` (a torch copy, read + write bytes) is kept beside them;
      * ``sclk_mhz_mfma_probe``: the shader clock measured in-kernel (cycle counter over the constant 100 MHz counter)
        under a dependent-MFMA loop on constant, low-entropy operands -- an upper bound: a GEMM on random data draws
        more power and the chip gives clock back (gate_up at M = 8192 ran at ~1.65 GHz effective under the profiler,
        profiles/r5_pmc_gemm4_vs_hipblaslt_gateup8192.txt); ``sclk_max_level`` from sysfs."""
    from .. import ops
    from ..models.weights import PackedLinear
    out: Dict[str, object] = {}
    n = 8192
    g = torch.Generator(device=device).manual_seed(1)
    x = torch.randn(n, n, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(n, n, device=device, generator=g) * 0.02).to(torch.bfloat16)
    pw = PackedLinear.from_dense(w, device)
    y = torch.empty(n, n, device=device, dtype=torch.bfloat16)
    e = ops.ext()

    def timed(fn, iters):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(device)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(iters):
            fn()
        ev1.record()
        torch.cuda.synchronize(device)
        return ev0.elapsed_time(ev1) / iters

    def gemm():
        e.gemm(x, pw.weight, n, n, y, ops.MODE_STORE, False, None, 1, None, -1.0, 0)

    flop = 2.0 * n * n * n
    ms = timed(gemm, 10)
    out["gemm_8192_tflops"] = round(flop / ms / 1e9, 1)
    # the clock under a full matrix load, measured in-kernel (shader cycles / 100 MHz real-time ticks over ~50 ms of
    # dependent MFMA chains on every CU; norm_embed.hip clock_probe_kernel) -- sysfs shows only the DPM request level
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    ticks = torch.zeros(3, dtype=torch.int64, device=device)
    e.clock_probe(200, 4 * cus, ticks)  # warm
    e.clock_probe(1000000, 4 * cus, ticks)
    torch.cuda.synchronize(device)
    cyc, rt = (int(v) for v in ticks[:2].tolist())
    if rt > 0:
        out["sclk_mhz_mfma_probe"] = round(cyc / rt * 100.0, 1)
    cur, top = _sclk_levels()
    if top is not None:
        out["sclk_max_level"] = top
    ms = timed(lambda: torch.mm(x, w.t(), out=y), 10)
    out["hipblaslt_8192_tflops"] = round(flop / ms / 1e9, 1)
    del x, w, pw, y
    src = torch.empty(1 << 29, dtype=torch.float32, device=device).fill_(1.0)  # 2 GiB
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    ms = timed(lambda: ext_prefetch(e, src, 4 * cus), 5)  # (cus: set above)
    out["stream_read_tbps"] = round(src.numel() * 4 / ms / 1e9, 2)
    # the decode kernels' own pattern: each wave one contiguous range, 1 KiB per instruction (norm_embed.hip
    # stream_probe_kernel; 8 workgroups per CU) -- the read rate a decode weight / KV stream can reach on this box
    ms = timed(lambda: ext_prefetch(e, src, -8 * cus), 5)
    out["stream_read_seq_tbps"] = round(src.numel() * 4 / ms / 1e9, 2)
    dst = torch.empty_like(src)
    ms = timed(lambda: dst.copy_(src), 5)
    out["copy_tbps"] = round(2 * src.numel() * 4 / ms / 1e9, 2)
    del src, dst
    torch.cuda.empty_cache()
    return out


def ext_prefetch(e, t: torch.Tensor, grid: int) -> None:
    e.prefetch(t, int(grid))
