#!/usr/bin/env python3
"""Headline benchmark: output tokens/s of LLaMA generation on MI355X (BASELINE.json metric).

One *step* = one full ``generate`` call on a batch of synthetic prompts: bf16 prefill of
``--prompt-len`` tokens, then ``--gen-len`` hipGraph-replayed greedy decode steps (EOS disabled so
every row produces every token; all work — prefill, every layer, lm_head, sampler, state update —
is inside the timed region). Weights are random-init with the exact architecture of ``--model``
(no checkpoints are available offline); the data are synthetic token ids.

Multi-GPU (torchrun, one process per GPU, RCCL): the world is split into ``world / tp``
data-parallel replicas of a ``tp``-way tensor-parallel model (default tp = 1: each GPU serves its
own batch -> weak scaling). ``value`` = total output tokens of all replicas / max-over-ranks time.

Extra keys (outside the timed region, reported alongside the headline):
  * ``latency_points``: decode ms/token at B = 1/8/32/64 (BASELINE.md protocol: prompt 128, cache for
    256 generated tokens, hipGraph replay, prefill excluded);
  * ``ttft``: time to first token of one ``--ttft-len`` (2048) token prompt at B = 1 (prefill of every layer with
    the flash-prefill attention + last-position lm_head + greedy token);
  * ``sampled``: tokens/s of whole ``generate`` calls in the reference's default sampling mode
    (temperature 0.8, top-p 0.95, top-k 50: jax_example.py:33, generation.py:22,34) at the headline batch;
  * ``tp_points`` (world > 1): the second half of the metric, tensor-parallel over every GPU of the job
    (MP = world): Llama-3-70B at MP 8 / 4 (README.md:52-53), Llama-2-13B at MP 2 (README.md:50); decode ms/token
    at B = 1/32/256 through the custom xGMI collectives, under a watchdog so a stuck collective can never cost the
    headline line;
  * ``tp_rank_proxy`` (one GPU): ONE rank of Llama-3-70B at MP 8 -- rank 0's shards at the real per-rank shapes
    (D 8192, 8 q / 1 kv heads, F 3584, V 16032, 80 layers, 17.6 GB), every per-token collective the same custom
    kernel on a world-1 instance (parallel/comm.py TPRankProxyComm): the per-rank decode step time, launch
    structure included, without the xGMI link's latency.

  python bench.py --gpus 1 --steps 3 --warmup 1
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --model llama3-70b --tp 8
"""
from __future__ import annotations

import argparse
import gc as _gc
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    # Serving-throughput operating point: 4096 concurrent sequences per replica (KV cache 103 GB of the 288 GB HBM; ~71
    # ms per decode step). Against 2048 on one box: 43.5k vs 41.5k tok/s -- the o / down / qkv projections fill the chip
    # without K splits at M = 4096 (profiles/r6_bench_batch_4096_vs_2048.jsonl); the prefill runs in two row chunks of
    # 2048 x 128 tokens (runtime/engine.py PREFILL_TOKENS). Latency points are reported separately.
    ap.add_argument("--batch", type=int, default=4096, help="sequences per replica")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=256)
    ap.add_argument("--layers", type=int, default=None, help="debug only: override layer count (INVALID for the metric)")
    ap.add_argument("--latency-batches", type=int, nargs="*", default=[1, 8, 32, 64])
    ap.add_argument("--no-sampled", action="store_true", help="skip the sampling-mode throughput point")
    ap.add_argument("--ttft-len", type=int, default=2048, help="prompt length of the time-to-first-token point "
                    "(B = 1; 0 = skip)")
    ap.add_argument("--tp-model", default="auto", help="model of the tensor-parallel points (world > 1); auto: "
                    "the BASELINE model of that MP degree (2: llama2-13b, 4/8: llama3-70b)")
    ap.add_argument("--tp-batches", type=int, nargs="*", default=[1, 32, 256])
    ap.add_argument("--tp-timeout", type=float, default=420.0, help="watchdog (s) of the tensor-parallel points")
    ap.add_argument("--proxy-model", default="llama3-70b", help="model of the one-GPU TP rank proxy ('' = skip)")
    ap.add_argument("--proxy-tp", type=int, default=8)
    ap.add_argument("--proxy-batches", type=int, nargs="*", default=[1, 32, 256])
    ap.add_argument("--mp1-model", default="llama3-70b", help="one-GPU (MP 1) decode point of this model at "
                    "--mp1-batch ('' = skip): all 80 layers of Llama-3-70B on one 288 GB GPU")
    ap.add_argument("--mp1-batch", type=int, default=256)
    ap.add_argument("--no-calibration", action="store_true")
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd import ops
    from jax_llama_amd.ops import autotune
    from jax_llama_amd.parallel import TPComm, init_distributed
    from jax_llama_amd.runtime import engine as eng_mod
    from jax_llama_amd.runtime.benchmark import (calibration, decode_latency, generate_tokens_per_sec,
                                                 time_to_first_token)
    from jax_llama_amd.runtime.engine import GenerationConfig, get_engine

    ctx = init_distributed()
    world = ctx.world
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ctx.setup_mesh(tp=args.tp)
    dev = ctx.device
    overrides = {} if args.layers is None else {"num_hidden_layers": args.layers}
    max_len = args.prompt_len + args.gen_len
    cfg = get_preset(args.model, max_seq_len=max(2048, max_len), **overrides)
    comm = TPComm.from_context(ctx, fused_hidden=cfg.hidden_size)
    model = LLaMAForCausalLM(cfg, device=dev, comm=comm, _do_init=False).init_random(seed=1234)
    torch.cuda.synchronize(dev)

    gen = torch.Generator().manual_seed(100 + ctx.dp_rank)
    prompts = torch.randint(3, cfg.vocab_size, (args.batch, args.prompt_len), generator=gen, dtype=torch.int32)
    gc = GenerationConfig(max_length=max_len, do_sample=False, pad_token_id=0, eos_token_id=-1)

    def step():
        return model.generate(prompts, generation_config=gc).sequences

    progress = _progress if ctx.rank == 0 else (lambda msg: None)
    t_start = time.perf_counter()
    for i in range(args.warmup):
        step()
        progress(f"warmup {i + 1}/{args.warmup} done ({time.perf_counter() - t_start:.1f} s)")
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step()
        progress(f"timed step {i + 1}/{args.steps} issued ({time.perf_counter() - t0:.1f} s)")
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ctx.barrier()
    torch.cuda.synchronize(dev)

    # time to first token on the already-captured engine (prefill + first sampled token)
    eng = get_engine(model, args.batch, max_len)
    torch.cuda.synchronize(dev)
    tp0 = time.perf_counter()
    eng.prefill_only(prompts, None, gc)
    torch.cuda.synchronize(dev)
    ttft = time.perf_counter() - tp0

    elapsed, ttft = ctx.all_reduce_max([elapsed, ttft])
    replicas = world // args.tp
    out_tokens = replicas * args.batch * args.gen_len * args.steps
    value = out_tokens / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    decode_ms_per_token = (ms_step - 1000.0 * ttft) / max(1, args.gen_len - 1)
    res = {
        "metric": "output_tokens_per_sec",
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak" if args.tp == 1 else "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic token ids, random-init weights (no checkpoints offline)",
        "config": {
            "model": args.model + ("" if args.layers is None else f"-{args.layers}L-DEBUG"),
            "global_batch": replicas * args.batch,
            "seq_len": max_len,
            "prompt_len": args.prompt_len,
            "gen_len": args.gen_len,
            "parallelism": f"dp{replicas}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
            "mp": args.tp,
        },
        "ttft_ms": round(1000.0 * ttft, 3),
        "decode_ms_per_token": round(decode_ms_per_token, 4),
        "decode_tokens_per_sec": round(replicas * args.batch * 1000.0 / decode_ms_per_token, 2),
        "weight_gb_per_gpu": round(model.weight_bytes() / 1e9, 3),
        "hbm_roofline_ms_per_token": round(model.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4),
    }
    del out, eng
    eng_mod._ENGINES.clear()  # free the headline batch's KV cache (103 GB at B = 4096) before the extra points
    torch.cuda.empty_cache()

    # The extra points never cost the headline line: each one's failure is recorded in its key instead. A failure
    # can be rank-local (OOM, one rank's comm.check()), so the ranks agree on every point's outcome before the next
    # one: once any rank failed, the remaining points are skipped on every rank (world > 1: they may be collective;
    # one process goes on with the next point).
    failed = {"any": False}

    def extra(key, fn):
        progress(f"side point {key} ...")
        ok = True
        if failed["any"]:
            res[key] = {"skipped": "an earlier extra point failed on some rank"}
            return
        try:
            fn()
        except Exception as ex:  # noqa: BLE001
            ok = False
            res[key] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        eng_mod._ENGINES.clear()
        torch.cuda.empty_cache()
        if world > 1:
            oks = [None] * world
            dist.all_gather_object(oks, ok)
            ok = all(oks)
        if not ok and world > 1:
            failed["any"] = True

    # ---- latency points (same model, BASELINE.md protocol)
    def latency_points():
        lat = []
        for b in args.latency_batches:
            lat.append(decode_latency(model, b, args.prompt_len, args.gen_len, seed=7, barrier=ctx.barrier))
        for p in lat:  # the slowest rank's number
            p["decode_ms_per_token"] = ctx.all_reduce_max([p["decode_ms_per_token"]])[0]
            p["decode_tokens_per_sec"] = round(p["batch"] * 1000.0 / p["decode_ms_per_token"], 2)
        res["latency_points"] = {"model": args.model, "mp": args.tp, "prompt_len": args.prompt_len,
                                 "cache_len": max_len, "points": lat}

    # ---- time to first token of one long prompt (prefill + first greedy token, B = 1)
    def ttft():
        t = time_to_first_token(model, 1, args.ttft_len, reps=3, seed=9, barrier=ctx.barrier)
        t["ttft_ms"] = ctx.all_reduce_max([t["ttft_ms"]])[0]
        t["prefill_tokens_per_sec"] = round(args.ttft_len * 1000.0 / t["ttft_ms"], 1)
        res["ttft"] = t

    # ---- sampling mode at the headline batch (reference default: T 0.8, top-p 0.95, top-k 50)
    def sampled():
        gcs = GenerationConfig(max_length=max_len, do_sample=True, temperature=0.8, top_p=0.95, top_k=50,
                               pad_token_id=0, eos_token_id=-1, seed=0)
        sp = generate_tokens_per_sec(model, args.batch, args.prompt_len, args.gen_len, gcs, seed=8,
                                     barrier=ctx.barrier)
        dt = ctx.all_reduce_max([sp["ms_per_generate"]])[0]
        res["sampled"] = {"temperature": 0.8, "top_p": 0.95, "top_k": 50, "batch_per_replica": args.batch,
                          "ms_per_generate": dt,
                          "tokens_per_sec": round(replicas * args.batch * args.gen_len * 1000.0 / dt, 2)}

    if args.latency_batches:
        extra("latency_points", latency_points)
    if args.ttft_len:
        extra("ttft", ttft)
    if not args.no_sampled:
        extra("sampled", sampled)
    if world == 1 and args.proxy_model and args.proxy_batches:
        extra("tp_rank_proxy", lambda: res.__setitem__("tp_rank_proxy", _tp_rank_proxy(args)))
    if world == 1 and args.mp1_model:
        del model
        # 141 GB of 70B weights: drop everything the earlier points left resident (engines, their KV caches, and
        # the grow-only op workspaces sized by the B = 2048 prefill's split-K slabs)
        eng_mod._ENGINES.clear()
        ops.workspace.clear()
        _gc.collect()
        torch.cuda.empty_cache()
        extra("mp1_point", lambda: res.__setitem__("mp1_point", _mp1_point(args)))
    if not args.no_calibration:  # last: the GEMM / copy probes of this box, next to the numbers above
        extra("calibration", lambda: res.__setitem__("calibration", calibration(dev)))
        _box_rooflines(res)
    res["gemm_plan_choice"] = {f"m{k[0]}_n{k[1]}_k{k[2]}_mode{k[3]}{'_rms' if k[4] else ''}": f"ks{v[0]}_tile{v[1]}"
                               for k, v in autotune.ksplit_table().items()}
    res["gemv_variant_choice"] = autotune.variant_table()

    # ---- tensor-parallel points: the BASELINE model of MP = world over every GPU of the job, under a watchdog
    if world > 1 and args.tp == 1 and args.tp_model and args.tp_batches and not failed["any"]:
        model = None
        torch.cuda.empty_cache()
        res["tp_points"] = _tp_points(args, ctx, res)

    if ctx.rank == 0:
        _emit(res, args.json_out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _box_rooflines(res):
    """Every ``hbm_roofline_ms_per_token`` (streamed bytes / the fixed 6.29 TB/s) gets a ``..._box`` twin divided by this
    box's own sequential read rate (calibration ``stream_read_seq_tbps``), so a point reads against its box."""
    tbps = (res.get("calibration") or {}).get("stream_read_seq_tbps")
    if not tbps:
        return
    for d in (res, res.get("tp_rank_proxy"), res.get("mp1_point")):
        if isinstance(d, dict) and "hbm_roofline_ms_per_token" in d:
            d["hbm_roofline_ms_per_token_box"] = round(d["hbm_roofline_ms_per_token"] * 6.29 / tbps, 4)


def _progress(msg: str) -> None:
    """A progress line on stderr (the one JSON result line stays alone on stdout): long phases -- a B = 4096 generate
    call takes ~24 s, the 70B points minutes -- never look hung to a watchdog on the job's output."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _emit(res, json_out):
    line = json.dumps(res)
    print(line, flush=True)
    if json_out:
        with open(json_out, "w") as f:
            f.write(line + "\n")


TP_MODEL_BY_MP = {2: "llama2-13b", 4: "llama3-70b", 8: "llama3-70b"}  # BASELINE.json configs 3 and 4


def _tp_rank_proxy(args):
    """One rank of ``--proxy-model`` at MP ``--proxy-tp`` on this GPU (``TPRankProxyComm``): decode ms/token at
    ``--proxy-batches`` next to the per-rank HBM roofline."""
    import torch

    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel import TPRankProxyComm
    from jax_llama_amd.runtime.benchmark import decode_latency

    cfg = get_preset(args.proxy_model, max_seq_len=max(2048, args.prompt_len + args.gen_len))
    comm = TPRankProxyComm.create(args.proxy_tp, fused_hidden=cfg.hidden_size)
    model = LLaMAForCausalLM(cfg, device="cuda", comm=comm, _do_init=False).init_random(seed=4321)
    out = {"model": args.proxy_model, "mp": args.proxy_tp, "rank": 0,
           "note": "one rank's shards and launches; collectives on a world-1 instance of the custom kernels "
                   "(no xGMI latency)",
           "prompt_len": args.prompt_len, "cache_len": args.prompt_len + args.gen_len,
           "weight_gb_per_gpu": round(model.weight_bytes() / 1e9, 3),
           "hbm_roofline_ms_per_token": round(model.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4),
           # qkv, attention, wo, w1|w3, w2 (+ the two all-reduce launches when the row-parallel GEMVs do not fuse them)
           "fused_row_parallel": comm.fused is not None}
    _progress("tp_rank_proxy: model ready")
    try:
        out["points"] = []
        for b in args.proxy_batches:
            out["points"].append(decode_latency(model, b, args.prompt_len, args.gen_len, seed=11))
            _progress(f"tp_rank_proxy: B = {b} done")
    finally:
        del model
        comm.close()
        torch.cuda.empty_cache()
    return out


def _mp1_point(args):
    """``--mp1-model`` (default Llama-3-70B, 141 GB of bf16 weights) on this one GPU: decode ms/token at
    ``--mp1-batch`` over the full generation window, next to its HBM roofline."""
    import torch

    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.runtime.benchmark import decode_latency

    cfg = get_preset(args.mp1_model, max_seq_len=max(2048, args.prompt_len + args.gen_len))
    resident_gb = round(torch.cuda.memory_allocated() / 1e9, 2)  # what the earlier points left allocated
    model = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).init_random(seed=77)
    _progress("mp1_point: model ready")
    try:
        p = decode_latency(model, args.mp1_batch, args.prompt_len, args.gen_len, seed=12)
        return {"model": args.mp1_model, "mp": 1, "weight_gb_per_gpu": round(model.weight_bytes() / 1e9, 3),
                "resident_gb_before_load": resident_gb,
                "hbm_roofline_ms_per_token": round(model.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4),
                "point": p}
    finally:
        del model
        torch.cuda.empty_cache()


def _tp_points(args, ctx, res):
    """The BASELINE model of MP = world (one TP group over every GPU). A watchdog thread ends the process with the
    headline line (and ``tp_points: timeout``) and a non-zero exit code if the phase does not finish in time."""
    import torch

    from jax_llama_amd.config import get_preset
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel import TPComm
    from jax_llama_amd.runtime.benchmark import decode_latency

    done = threading.Event()

    def watchdog():
        if not done.wait(args.tp_timeout):
            if ctx.rank == 0:
                res["tp_points"] = {"status": "timeout", "timeout_s": args.tp_timeout}
                _emit(res, args.json_out)
            sys.stdout.flush()
            os._exit(3)  # the headline line is out, but a stuck phase is not a clean run

    threading.Thread(target=watchdog, daemon=True).start()
    world = ctx.world
    tp_model = TP_MODEL_BY_MP.get(world, "llama3-70b") if args.tp_model == "auto" else args.tp_model
    out = {"model": tp_model, "mp": world, "prompt_len": args.prompt_len, "cache_len":
           args.prompt_len + args.gen_len}
    try:
        ctx.setup_mesh(tp=world)
        cfg = get_preset(tp_model, max_seq_len=max(2048, args.prompt_len + args.gen_len))
        comm = TPComm.from_context(ctx, fused_hidden=cfg.hidden_size)
        out["custom_allreduce"] = comm.custom is not None
        out["fused_row_parallel"] = comm.fused is not None
        out["litmus"] = comm.litmus()  # the paths verified on these links before use (else RCCL carries them)
        model = LLaMAForCausalLM(cfg, device=ctx.device, comm=comm, _do_init=False).init_random(seed=4321)
        out["weight_gb_per_gpu"] = round(model.weight_bytes() / 1e9, 3)
        out["hbm_roofline_ms_per_token"] = round(model.streamed_weight_bytes_per_token() / 6.29e12 * 1e3, 4)
        pts = []
        for b in args.tp_batches:
            p = decode_latency(model, b, args.prompt_len, args.gen_len, seed=9, barrier=ctx.barrier)
            p["decode_ms_per_token"] = ctx.all_reduce_max([p["decode_ms_per_token"]])[0]
            p["decode_tokens_per_sec"] = round(b * 1000.0 / p["decode_ms_per_token"], 2)
            pts.append(p)
        out["points"] = pts
        out["status"] = "ok"
        del model
        torch.cuda.empty_cache()
    except Exception as ex:  # reported, never fatal to the headline line
        out["status"] = f"error: {type(ex).__name__}: {str(ex)[:300]}"
    done.set()
    return out


if __name__ == "__main__":
    main()
