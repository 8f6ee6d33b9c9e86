"""Tensor-parallel model on the GPU kernels: 2 ranks sharing the test box's one GPU (a gloo group
for the handle exchange and gathers, the custom IPC all-reduce for the row-parallel sums) must
reproduce the single-process GPU model: logits and greedy generation. On an 8-GPU node the same
code runs one rank per GPU over RCCL + xGMI."""
from __future__ import annotations

import multiprocessing as mp
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0", JLA_NO_GRAPH="1")
        import torch.distributed as dist
        from helpers import build, gpu_config, left_padded_batch, rel_err
        from jax_llama_amd.models import LLaMAForCausalLM
        from jax_llama_amd.parallel import TPComm, init_distributed
        from jax_llama_amd.runtime.engine import GenerationConfig
        ctx = init_distributed(backend="gloo", device_type="cuda")
        ctx.setup_mesh(tp=world)
        comm = TPComm.from_context(ctx)
        assert comm.custom is not None, "custom all-reduce not created"
        cfg = gpu_config(num_attention_heads=4, num_key_value_heads=2, hidden_size=512, intermediate_size=1024,
                         vocab_size=512)
        _, _, _, params = build(cfg, seed=21)
        tp_model = LLaMAForCausalLM(cfg, device="cuda", comm=comm).load_params(params)
        ref = LLaMAForCausalLM(cfg, device="cuda").load_params(params)
        toks, mask = left_padded_batch([5, 9, 12], 12, cfg.vocab_size, pad=2, seed=4)
        pos = mask.cumsum(-1) - 1
        lt = tp_model(toks, attention_mask=mask, position_ids=pos).logits.float().cpu()
        lr = ref(toks, attention_mask=mask, position_ids=pos).logits.float().cpu()
        m = mask.bool()
        err = rel_err(lt[m], lr[m])
        gc = GenerationConfig(max_length=28, do_sample=False, pad_token_id=2, eos_token_id=-1)
        st = tp_model.generate(toks, attention_mask=mask, generation_config=gc).sequences.cpu()
        sr = ref.generate(toks, attention_mask=mask, generation_config=gc).sequences.cpu()
        gcs = GenerationConfig(max_length=28, do_sample=True, temperature=0.8, top_p=0.9, pad_token_id=2,
                               eos_token_id=-1, seed=5)
        ss = tp_model.generate(toks, attention_mask=mask, generation_config=gcs).sequences.cpu()
        car_err = comm.custom.error()
        dist.barrier()
        q.put(("ok", rank, (err, torch.equal(st, sr), ss.tolist(), car_err)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - surfaced in the parent
        import traceback
        q.put(("err", rank, traceback.format_exc()))


@pytest.mark.timeout(400)
def test_tp2_gpu_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = []
    try:
        for _ in range(world):
            outs.append(q.get(timeout=360))
    finally:
        for p in procs:
            p.join(timeout=60)
    for status, rank, payload in outs:
        assert status == "ok", payload
    res = {rank: payload for _, rank, payload in outs}
    for r in range(world):
        err, greedy_equal, sampled, car_err = res[r]
        assert err < 2e-2, err
        assert greedy_equal
        assert car_err == 0
    assert res[0][2] == res[1][2]  # every rank sampled the same tokens
