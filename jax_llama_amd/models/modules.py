"""Decoder building blocks with the reference's module structure.

Reference (``/root/reference/jax_llama/model.py``): ``FlaxLLaMAAttention`` (:105-300),
``FlaxLLaMAMLP`` (:302-340), ``FlaxLLaMABlock`` (:342-400), ``FlaxLLaMABlockCollection`` (:548-600).
Here each block is a thin, stateless view over one layer's packed weights that issues the fused
MI355X ops -- the parameters live in ``LLaMAForCausalLM.layers`` so TP sharding, the packed MFMA
layout and hipGraph capture see one flat set of tensors:

  attention: [RMSNorm folded] qkv GEMV/GEMM + RoPE + KV-cache write (one kernel in decode), cache
             attention (split-KV decode / flash prefill, GQA by indexing), wo with the residual add
             fused into its epilogue (+ TP all-reduce); at small batch qkv + attention (+ wo) are one
             launch                                                          -- model.py:383-392
  mlp:       [RMSNorm folded] w1|w3 GEMV/GEMM with SiLU*up epilogue, w2 with the residual add
             (+ TP all-reduce)                                               -- model.py:394-398

The residual stream is ``h`` (fp32) plus its bf16 mirror ``hb`` (the A operand of the next
projection, written by the residual epilogues).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .. import ops
from ..ops import reference as ref


class LLaMAAttention:
    def __init__(self, model, layer_idx: int):
        self.model = model
        self.layer_idx = layer_idx

    @property
    def weights(self):
        return self.model.layers[self.layer_idx]

    def __call__(self, h, hb, positions, cache, slot0, kv_start, key_mask, seq_len: int,
                 output_attentions: bool = False, pk: Optional["PackedActs"] = None) -> Optional[torch.Tensor]:
        m, lw = self.model, self.weights
        kc, vc = cache.layer(self.layer_idx)
        splits = og = 0
        o_state = None
        if not output_attentions:
            # the o projection in the same launch where it fits (the 70B tensor-parallel shard at small batch)
            og = ops.qkv_attention_o_groups(hb, lw.o, m.n_heads, m.n_kv_heads) if seq_len == 1 else 0
            o_state = m.comm.fused_o_state(hb, lw.o) if og else None
            og = og if o_state is not None else 0
            splits = ops.qkv_attention_splits(hb, lw.qkv, kc, seq_len, m.n_heads, m.n_kv_heads, key_mask, og)
            if og and not splits:
                og = 0
                splits = ops.qkv_attention_splits(hb, lw.qkv, kc, seq_len, m.n_heads, m.n_kv_heads, key_mask)
        if splits:  # small-batch decode: qkv projection + attention (+ o projection) in one launch
            hb_p = pk.hb if pk else None
            o = (lw.o, h, hb, hb_p, o_state) if og else None
            att_p = pk.att if pk is not None and not og else None
            a = ops.linear_qkv_attention(hb, lw.qkv, m.eps, m.rope, positions, kc, vc, slot0, kv_start, m.n_heads,
                                         m.n_kv_heads, m.head_dim, splits, x_packed=pk.hb_in() if pk else None,
                                         out_packed=att_p, o=o)
            if not og:
                m._row_parallel(a, lw.o, h, hb, x_packed=att_p, mirror_packed=hb_p)
            if pk is not None and pk.hb is not None:
                pk.hb_ok = True
            return None
        q = ops.linear_qkv_rope(hb, lw.qkv, m.eps, m.rope, positions, kc, vc, slot0, seq_len,
                                m.n_heads, m.n_kv_heads, m.head_dim, x_packed=pk.hb_in() if pk else None)
        b = hb.shape[0] // seq_len
        q4 = q.reshape(b, seq_len, m.n_heads, m.head_dim)
        weights = None
        att_p = None
        if output_attentions:
            # the layer output still comes from the attention kernel (as without the flag); the softmax weights the
            # reference returns (:277-286) are materialised beside it by the fp32 oracle, on the tensors' device
            s0 = int(slot0) if not torch.is_tensor(slot0) else int(slot0.item())
            _, weights = ref.attention(q4, kc, vc, s0, kv_start, key_mask, return_weights=True)
            a = ops.attention(q4, kc, vc, slot0, kv_start, key_mask)
        else:
            att_p = pk.att if pk is not None and ops.attention_packs(q4, kc, key_mask) else None
            a = ops.attention(q4, kc, vc, slot0, kv_start, key_mask, out_packed=att_p)
        m._row_parallel(a, lw.o, h, hb, x_packed=att_p, mirror_packed=pk.hb if pk else None)
        if pk is not None and pk.hb is not None:
            pk.hb_ok = True
        return weights


class LLaMAMLP:
    def __init__(self, model, layer_idx: int):
        self.model = model
        self.layer_idx = layer_idx

    def __call__(self, h, hb, pk: Optional["PackedActs"] = None) -> None:
        m, lw = self.model, self.model.layers[self.layer_idx]
        g = ops.linear_swiglu(hb, lw.gu, rms_eps=m.eps, x_packed=pk.hb_in() if pk else None,
                              out_packed=pk.act if pk else None)

        m._row_parallel(g, lw.down, h, hb, x_packed=pk.act if pk else None, mirror_packed=pk.hb if pk else None)


class LLaMABlock:
    """Pre-norm block: ``h += attn(norm(h)); h += mlp(norm(h))``."""

    def __init__(self, model, layer_idx: int):
        self.attention = LLaMAAttention(model, layer_idx)
        self.feed_forward = LLaMAMLP(model, layer_idx)

    def __call__(self, h, hb, positions, cache, slot0, kv_start, key_mask, seq_len: int,
                 output_attentions: bool = False, pk: Optional["PackedActs"] = None):
        w = self.attention(h, hb, positions, cache, slot0, kv_start, key_mask, seq_len, output_attentions, pk)
        self.feed_forward(h, hb, pk)
        return w


class PackedActs:
    """Packed-layout copies (ops.packed_rows x cols, csrc/kernels/common.h pack_off) of the decode activations
    that feed a projection: the residual mirror hb (written by the wo / w2 epilogues, read by wqkv and w1|w3),
    the attention output (read by wo) and the SwiGLU output (read by w2). hb has no packed copy before the first
    residual epilogue of the step (the embedding writes only the row-major mirror)."""

    def __init__(self, rows: int, model, device, full: bool = True):
        # full = False (rows above ops.PACKED_X_MAX_M): only the attention output is packed (wo reads it); hb / the
        # SwiGLU output stay row-major (profiles/r2_packed_x_decode_ab.jsonl). Since the tiled split-K GEMM's reduce
        # epilogue writes packed copies too, full packing reaches 64 rows (profiles/r3_packed_x_m64_ab.jsonl)
        self.hb = ops.packed_empty(rows, model.config.hidden_size, device) if full else None
        self.att = ops.packed_empty(rows, model.n_heads * model.head_dim, device)
        self.act = ops.packed_empty(rows, model.ffn, device) if full else None
        self.hb_ok = False

    def hb_in(self) -> Optional[torch.Tensor]:
        return self.hb if self.hb_ok else None


class LLaMABlockCollection:
    """The layer loop (reference :579-595). Inside a hipGraph-captured decode step this loop is
    recorded once and replayed per token."""

    def __init__(self, model):
        self.blocks: List[LLaMABlock] = [LLaMABlock(model, i) for i in range(len(model.layers))]
        self.model = model

    def __len__(self):
        return len(self.blocks)

    def __call__(self, h, hb, positions, cache, slot0, kv_start, key_mask, seq_len: int,
                 output_hidden_states: bool = False, output_attentions: bool = False):
        hidden, attns = [], []
        b = hb.shape[0] // seq_len
        rows = hb.shape[0]
        pk = None
        if (ops.PACKED_X and hb.is_cuda and ops.PACKED_X_MIN_M <= rows <= min(ops.PACKED_ATT_MAX_M, ops.SKINNY_M)
                and self.model.comm.packs_residual(rows * self.model.config.hidden_size * 4)):
            # TP: the residual all-reduce writes the packed hb copy (csrc/kernels/allreduce.hip car_epilogue)
            pk = PackedActs(rows, self.model, hb.device, full=rows <= ops.PACKED_X_MAX_M)
        for blk in self.blocks:
            if output_hidden_states:
                hidden.append(h.reshape(b, seq_len, -1).clone())
            w = blk(h, hb, positions, cache, slot0, kv_start, key_mask, seq_len, output_attentions, pk)
            if output_attentions:
                attns.append(w)
        return hidden, attns
