#!/usr/bin/env python3
"""Latency of the custom xGMI collectives (csrc/kernels/allreduce.hip) vs message size.

  python tools/bench_allreduce.py --world 8 [--sizes-kib 16 64 ...] [--out gpurun_out/car.jsonl]

Spawns ``--world`` processes. On a one-GPU box they all share GPU 0 (``--share``, the default when
fewer GPUs than ranks are visible): the numbers then measure the protocol (launch, flag round trips,
local HBM traffic) rather than xGMI link speed. On an 8-GPU node each rank gets its own GPU.
Each size is timed as a hipGraph of ``--reps`` back-to-back calls (what a decode step sees), for the
fused residual all-reduce (bf16 partial -> fp32 h + bf16 mirror) one-shot and two-shot.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, args, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    n_dev = torch.cuda.device_count()
    torch.cuda.set_device(0 if args.share or n_dev < world else rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
    car = CustomAllReduce.create_for(rank, world, None, max_bytes=max(args.sizes_kib) * 1024)
    rows = []
    for kib in args.sizes_kib:
        n = kib * 1024 // 2
        x = torch.randn(n, device="cuda").to(torch.bfloat16)
        h = torch.zeros(n, device="cuda")
        hb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        for ts in ((False, True) if world >= 2 else (False,)):
            car.all_reduce_residual_(x, h, hb, two_shot=ts)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(args.reps):
                    car.all_reduce_residual_(x, h, hb, two_shot=ts)
            g.replay()
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / (args.iters * args.reps)
            t = torch.tensor([us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            rows.append({"op": "allreduce_residual_bf16", "world": world, "kib_per_rank": kib,
                         "two_shot": ts, "us_per_call": round(float(t), 2),
                         "shared_gpu": bool(args.share or n_dev < world)})
    err = car.error()
    car.close()
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put((rows, err))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--sizes-kib", type=int, nargs="+", default=[16, 64, 256, 1024, 4096, 8192])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--share", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    rows, err = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    for r in rows:
        r["error_word"] = err
        line = json.dumps(r)
        print(line, flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
