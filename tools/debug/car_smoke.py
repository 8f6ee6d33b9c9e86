"""Debug driver for the custom all-reduce: 2 processes on GPU 0, step-by-step prints."""
import multiprocessing as mp
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jax_llama_amd import ops
    e = ops.ext()
    print(rank, "alloc", flush=True)
    buf, sig, hb, hs = e.car_alloc(1 << 20, world)
    print(rank, "alloc ok", hex(buf), hex(sig), len(hb), flush=True)
    handles = [None] * world
    dist.all_gather_object(handles, (bytes(hb), bytes(hs)))
    print(rank, "gathered", flush=True)
    st = e.car_init(rank, world, 1 << 20, buf, sig, [h[0] for h in handles], [h[1] for h in handles])
    print(rank, "init ok", flush=True)
    dist.barrier()
    x = torch.full((1024,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    e.car_allreduce(st, x, y)
    torch.cuda.synchronize()
    print(rank, "result", y[:4].tolist(), "err", e.car_error(st), flush=True)
    dist.barrier()
    from jax_llama_amd.parallel.custom_allreduce import CustomAllReduce
    car = CustomAllReduce.create_for(rank, world, None, max_bytes=8 << 20)
    print(rank, "created", flush=True)
    for n, dt in [(8, torch.float32), (4096, torch.bfloat16), (300_000, torch.float32), (512 * 4096, torch.bfloat16)]:
        x = torch.ones(n, dtype=dt, device="cuda") * (rank + 1)
        y = car.all_reduce(x)
        torch.cuda.synchronize()
        print(rank, n, dt, float(y.float().min()), float(y.float().max()), flush=True)
    buf = torch.ones(16384, dtype=torch.bfloat16, device="cuda")
    car.all_reduce_(buf.clone())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        car.all_reduce_(buf)
    print(rank, "captured", flush=True)
    buf.fill_(rank + 1)
    g.replay()
    torch.cuda.synchronize()
    print(rank, "graph", float(buf.float().min()), float(buf.float().max()), car.error(), flush=True)
    dist.barrier()
    car.close()
    print(rank, "closed", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    print(rank, "done", flush=True)


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, 2, 29533)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    print("exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if all(p.exitcode == 0 for p in ps) else 1)
