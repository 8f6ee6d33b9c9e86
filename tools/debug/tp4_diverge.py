"""Debug: where do the TP-4 greedy sequences (graph / eager) diverge from the TP-1 reference?"""
import multiprocessing as mp
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    from helpers import left_padded_batch
    from jax_llama_amd.models import LLaMAForCausalLM
    from jax_llama_amd.parallel import TPComm, init_distributed
    from jax_llama_amd.runtime.engine import DecodeEngine, GenerationConfig
    from test_tp_gpu import _config, _gpu_params
    ctx = init_distributed(backend="gloo", device_type="cuda")
    ctx.setup_mesh(tp=world)
    comm = TPComm.from_context(ctx, reduce_dtype=torch.float32)
    cfg = _config("70b")
    params = _gpu_params(cfg, seed=21)
    m = LLaMAForCausalLM(cfg, device="cuda", comm=comm, _do_init=False).load_params(params)
    toks, mask = left_padded_batch([5, 9, 12, 12], 12, cfg.vocab_size, pad=2, seed=4)
    gc = GenerationConfig(max_length=28, do_sample=False, pad_token_id=2, eos_token_id=-1)
    outs = {}
    for g in (True, False, True):
        e = DecodeEngine(m, 4, 28, use_graph=g)
        outs.setdefault(g, []).append(e.run(toks, mask, gc).cpu().clone())
        del e
    del m
    torch.cuda.empty_cache()
    dist.barrier()
    if rank == 0:
        ref = LLaMAForCausalLM(cfg, device="cuda", _do_init=False).load_params(params)
        sr = ref.generate(toks, attention_mask=mask, generation_config=gc).sequences.cpu()
        for g, lst in outs.items():
            for i, s in enumerate(lst):
                d = (s != sr).nonzero().tolist()
                print("graph" if g else "eager", i, "diff vs tp1:", d[:6], flush=True)
        print("graph runs equal:", torch.equal(outs[True][0], outs[True][1]), "graph==eager:",
              torch.equal(outs[True][0], outs[False][0]), flush=True)
    dist.barrier()
    q.put(rank)


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    for _ in ps:
        q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
