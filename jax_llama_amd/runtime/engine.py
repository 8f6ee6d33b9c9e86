"""Generation engine: prefill + hipGraph-replayed decode steps.

Semantics follow HF ``FlaxGenerationMixin.generate`` (transformers<5), which the reference
inherits (``generation.py:28-41`` builds the ``GenerationConfig``):

  * ``sequences = full((B, max_length), pad)``; the prompt occupies ``[:, :S]``;
  * the prefill is the first loop-body call, then the decode loop runs while
    ``cur_len < max_length`` and not every row has produced ``eos``;
  * a finished row emits ``pad``; ``is_sent_finished |= next == eos``;
  * greedy = ``argmax`` (first max); sampling = temperature -> top-k (default 50) -> top-p ->
    categorical;
  * positions: ``cumsum(mask) - 1`` for the prompt, then ``last + 1`` per step
    (``model.py:758, 771``).

MI355X execution model (replaces XLA's compiled ``lax.while_loop``):
  * the whole decode step (embedding, all layers, lm_head, sampler, state update) reads its
    inputs — token ids, positions, the cache slot, ``cur_len`` and the finished flags — from
    device buffers and writes the next state back, so it is captured ONCE into a hipGraph
    (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replayed per token with no host
    work besides the launch;
  * the host polls the finished flags only every ``check_every`` steps (rows that finished
    earlier keep emitting ``pad``, so polling late never changes the output).
"""
from __future__ import annotations

import dataclasses
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Optional

import torch

from .. import ops
from ..ops import reference as ref

_NEG_INF = float("-inf")


@dataclass
class GenerationConfig:
    """Subset of HF ``GenerationConfig`` used by the reference (``generation.py:32-40``)."""

    max_length: Optional[int] = None
    max_new_tokens: Optional[int] = None
    do_sample: bool = False
    temperature: float = 1.0
    top_k: int = 50  # HF default; the reference never overrides it
    top_p: float = 1.0
    num_beams: int = 1
    pad_token_id: Optional[int] = None
    eos_token_id: Optional[int] = None
    seed: int = 0


# prompt tokens per prefill forward (DecodeEngine._prefill_rows): larger batches run their prefill in row chunks
PREFILL_TOKENS = int(os.environ.get("JLA_PREFILL_TOKENS", str(1 << 18)))

# greedy decoding takes the argmax inside the lm_head GEMM epilogue (JLA_FUSED_ARGMAX=0: logits + argmax)
FUSED_GREEDY = os.environ.get("JLA_FUSED_ARGMAX", "1") != "0"


def _fused_greedy() -> bool:
    return FUSED_GREEDY


@dataclass
class GenerateOutput:
    sequences: torch.Tensor


# --------------------------------------------------------------------------------------
# Sampling
# --------------------------------------------------------------------------------------
def _greedy(model, logits_local) -> torch.Tensor:
    """``logits_local``: this rank's ``[B, V/tp]`` logits, or its already reduced ``(idx, val)``
    (``forward_tokens(logits_mode="argmax")``: argmax fused into the lm_head GEMM). Under TP the
    per-rank ``(max, argmax)`` pairs are reduced by one custom gather kernel (``comm.argmax``)."""
    if isinstance(logits_local, tuple):
        (idx, val), v_local = logits_local, model.vocab_local
    else:
        (idx, val), v_local = ops.argmax(logits_local), logits_local.shape[1]
    return model.comm.argmax(val, idx, v_local)


def _sample(model, logits_local: torch.Tensor, gc: GenerationConfig, gen: Optional[torch.Generator],
            step: Optional[torch.Tensor] = None):
    """temperature -> top-k -> top-p -> categorical (Gumbel-max), exact under vocab sharding.

    top_k in [1, 64] (HF default 50): the on-device sampler (ops.topk_sample: radix-select top-k
    kernels + Philox Gumbel-max keyed by (seed, step)), graph-capturable and identical on CPU.
    Otherwise (top_k = 0 / > 64): torch sort path."""
    comm = model.comm
    v_local = logits_local.shape[1]
    k = min(gc.top_k or 0, v_local * comm.size)
    if step is not None and 1 <= k <= ops.SAMPLER_MAX_K and gc.temperature and gc.temperature > 0:
        if logits_local.device.type == "cpu" or ops.ext().topk_chunks(v_local) * min(k, v_local) <= 4096:
            return ops.topk_sample(logits_local.float().contiguous(), k, gc.temperature, gc.top_p,
                                   gc.seed, step, comm if comm.size > 1 else None)
    x = logits_local.float()
    if gc.temperature is not None and gc.temperature != 1.0:
        x = x / gc.temperature
    if gc.top_k:
        k = min(gc.top_k, x.shape[1])
        vals, idx = torch.topk(x, k, dim=-1)
        idx = (idx + comm.rank * x.shape[1]).to(torch.int32)
        if comm.size > 1:
            gv, gi = comm.gather_topk(vals.contiguous(), idx.contiguous())
            vals, sel = torch.topk(gv, k, dim=-1)
            idx = gi.gather(1, sel)
    else:
        full = model.gather_logits(x)
        vals, idx = torch.sort(full, dim=-1, descending=True)
    if gc.top_p is not None and gc.top_p < 1.0:
        # vals are sorted descending (topk returns sorted)
        probs = torch.softmax(vals, -1)
        cum = probs.cumsum(-1)
        keep = torch.roll(cum < gc.top_p, 1, dims=-1)
        keep[:, 0] = True
        vals = torch.where(keep, vals, torch.full_like(vals, _NEG_INF))
    u = torch.rand(vals.shape, device=vals.device, generator=gen, dtype=torch.float32)
    gumbel = -torch.log(-torch.log(u.clamp_min(1e-20)).clamp_min(1e-20))
    choice = (vals + gumbel).argmax(-1)
    return idx.gather(1, choice[:, None]).squeeze(1).to(torch.int32)


# --------------------------------------------------------------------------------------
class DecodeEngine:
    """Owns the KV cache and the device-resident decode state for one (B, max_length)."""

    def __init__(self, model, batch_size: int, max_length: int, use_graph: Optional[bool] = None,
                 check_every: int = 16):
        self.model = model
        self.b = batch_size
        self.max_length = max_length
        dev = model.device
        self.device = dev
        if use_graph is None:
            use_graph = dev.type == "cuda" and os.environ.get("JLA_NO_GRAPH", "0") != "1"
        self.use_graph = use_graph
        self.check_every = check_every
        self.cache = model.init_cache(batch_size, max_length)
        i32 = dict(dtype=torch.int32, device=dev)
        self.tokens = torch.zeros(batch_size, 1, **i32)
        self.positions = torch.zeros(batch_size, 1, **i32)
        self.kv_start = torch.zeros(batch_size, **i32)
        self.finished = torch.zeros(batch_size, **i32)
        self.cur_len = torch.zeros(1, **i32)
        self.sequences = torch.zeros(batch_size, max_length, **i32)
        self.key_mask: Optional[torch.Tensor] = None
        self._graph = None
        self._graph_key = None
        self.keep_graph = False  # keep the captured graph's topology (runtime/benchmark.py counts its kernel nodes)
        self._gen: Optional[torch.Generator] = None
        self.gc: Optional[GenerationConfig] = None

    # ---------------------------------------------------------------------------------
    def _next_token(self, logits_local):
        if self.gc.do_sample:
            return _sample(self.model, logits_local, self.gc, self._gen, self.cur_len)
        return _greedy(self.model, logits_local)

    def _update(self, nxt: torch.Tensor):
        """Device-side HF loop-body bookkeeping (pad for finished rows, eos tracking,
        sequences write, position/slot/cur_len advance)."""
        if self.device.type == "cuda":
            ops.ext().decode_update(nxt, self.finished, self.sequences, self.cur_len, self.tokens,
                                    self.positions, self.cache.index_t, int(self.gc.pad_token_id),
                                    int(self.gc.eos_token_id))
            return
        fin = self.finished.bool()
        nxt = torch.where(fin, torch.full_like(nxt, self.gc.pad_token_id), nxt)
        self.finished.copy_((fin | (nxt == self.gc.eos_token_id)).to(torch.int32))
        cl = int(self.cur_len.item())
        if cl < self.max_length:
            self.sequences[:, cl] = nxt
        self.tokens[:, 0] = nxt
        self.positions.add_(1)
        self.cache.index_t.add_(1)
        self.cur_len.add_(1)

    def _logits_mode(self) -> str:
        return "argmax" if _fused_greedy() and not self.gc.do_sample else "last"

    def _decode_step(self):
        logits, *_ = self.model.forward_tokens(self.tokens, self.positions, self.cache, self.cache.index_t,
                                               self.kv_start, self.key_mask, logits_mode=self._logits_mode())
        self._update(self._next_token(logits))

    # ---------------------------------------------------------------------------------
    def prefill(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor]):
        model, dev = self.model, self.device
        ids = input_ids.to(dev, torch.int32)
        b, s = ids.shape
        assert b == self.b and s < self.max_length
        if attention_mask is None:
            mask = torch.ones(b, s, dtype=torch.int32)
        else:
            mask = attention_mask.to("cpu", torch.int32)
        positions = (mask.cumsum(-1) - 1).to(torch.int32)
        ext_mask = torch.ones(b, self.max_length, dtype=torch.int32)
        ext_mask[:, :s] = mask
        from ..models.llama import mask_to_kv_start
        kv_start, key_mask = mask_to_kv_start(ext_mask, dev)
        self.kv_start.copy_(kv_start)
        self.key_mask = key_mask
        self.cache.reset()
        self.sequences.fill_(self.gc.pad_token_id)
        self.sequences[:, :s] = ids
        self.finished.zero_()
        pos_dev = positions.to(dev)
        logits = self._prefill_rows(ids, pos_dev)
        self.cache.advance(s)
        # state for the loop body: cur_len = S (also the sampler's Philox step), token/pos of the
        # last prompt position
        self.cur_len.fill_(s)
        nxt = self._next_token(logits)
        self.positions.copy_(pos_dev[:, -1:])
        # _update writes sequences[:, S], advances pos (+1), slot (+1 -> S+1 ... ) and cur_len.
        # The prefill already advanced the slot by S; undo the update's +1 on the slot.
        self.cache.index_t.sub_(1)
        self._update(nxt)
        self.cache.index = s  # host mirror (decode steps track the slot on the device)
        return s + 1

    def _prefill_rows(self, ids: torch.Tensor, pos_dev: torch.Tensor):
        """The prompt forward, in row chunks of at most PREFILL_TOKENS tokens: every kernel then sees at most the
        token count the GEMMs already saturate the chip with (M = 262144: 2048 rows x 128), whatever the batch, and no
        activation index of a larger batch can pass 2^31 elements. One chunk up to that size (the common case)."""
        b, s = ids.shape
        rows = max(1, PREFILL_TOKENS // max(1, s))
        mode = self._logits_mode()
        if b <= rows:
            logits, *_ = self.model.forward_tokens(ids, pos_dev, self.cache, 0, self.kv_start, self.key_mask,
                                                   logits_mode=mode)
            return logits
        parts = []
        for b0 in range(0, b, rows):
            b1 = min(b, b0 + rows)
            km = self.key_mask[b0:b1] if self.key_mask is not None else None
            lg, *_ = self.model.forward_tokens(ids[b0:b1], pos_dev[b0:b1], self.cache.rows(b0, b1), 0,
                                               self.kv_start[b0:b1], km, logits_mode=mode)
            parts.append(lg)
        if isinstance(parts[0], tuple):  # greedy: (idx, val) per chunk
            return tuple(torch.cat([p[i] for p in parts]) for i in range(len(parts[0])))
        return torch.cat(parts)

    def prefill_only(self, input_ids, attention_mask, gc: GenerationConfig) -> int:
        """Prefill + first token only (time-to-first-token measurement)."""
        self.gc = gc
        return self.prefill(input_ids, attention_mask)

    def _graph_state(self):
        # the graph records buffer addresses: the scratch workspaces (ops.workspace) and the sampling mode
        return (self.gc.do_sample, self.key_mask is not None, ops.workspace.generation, _fused_greedy(),
                ops.ARGMAX_FUSED_MIN_M, ops.SKINNY_ARGMAX, ops.QKV_ATTN, self.model.comm.reduce_dtype)

    def _ensure_graph(self):
        if self._graph is not None and self._graph_key == self._graph_state():
            return
        for _ in range(3):
            key = self._graph_state()
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph(keep_graph=self.keep_graph)
            # Capture records kernels without executing them; state buffers are static.
            with torch.cuda.graph(g):
                self._decode_step()
            self._graph, self._graph_key = g, key
            if self._graph_state() == key:  # no workspace grew while capturing
                return
        raise RuntimeError("decode graph capture keeps reallocating workspaces")

    def _poll(self) -> bool:
        """Host poll (every ``check_every`` steps): True once every row has finished. Also raises if a
        custom TP collective gave up waiting for a peer."""
        done = bool(self.finished.all().item())
        self._check()
        return done

    def _check(self):
        """Device-side failure words: a custom TP collective that gave up on a peer (comm.check), an in-launch wait
        that timed out (ops.check_inlaunch: the fused qkv + attention launch), out-of-range indices (debug build)."""
        self.model.comm.check()
        if self.device.type == "cuda":
            ops.check_inlaunch()
        ops.check_bounds()  # bounds-checked debug build only (JLA_DEBUG_BOUNDS=1): out-of-range device indices

    def run(self, input_ids, attention_mask, gc: GenerationConfig) -> torch.Tensor:
        self.gc = gc
        rng_saved = None
        if gc.do_sample:
            self._gen = torch.Generator(device=self.device)
            self._gen.manual_seed(int(gc.seed))
            if self.use_graph:
                # The on-device sampler (ops.topk_sample, top_k <= 64) draws from its own Philox stream keyed by
                # (seed, step) and touches no torch RNG. The torch fallback (top_k = 0 or > 64) under graph capture
                # needs the device's default generator (graph-safe philox offsets): seed it for this call and give
                # the caller's RNG state back afterwards.
                self._gen = None
                if self.device.type == "cuda":
                    rng_saved = torch.cuda.get_rng_state(self.device)
                    torch.cuda.manual_seed(int(gc.seed))
        try:
            return self._run(input_ids, attention_mask)
        except Exception:
            # a failed step (a peer or in-launch timeout, an error mid-decode) can leave non-finite rows in this
            # engine's cache beyond where the next prompt writes; the kernels mask keys past the valid length by
            # probability 0, and 0 x NaN is NaN: zero the cache so the next call starts as from a fresh engine
            self.cache.k.zero_()
            self.cache.v.zero_()
            raise
        finally:
            if rng_saved is not None:
                torch.cuda.set_rng_state(rng_saved, self.device)

    def _run(self, input_ids, attention_mask) -> torch.Tensor:
        cur = self.prefill(input_ids, attention_mask)
        steps_left = self.max_length - cur
        done = steps_left <= 0
        first = True
        step = 0
        while not done:
            if self.use_graph and not first:
                self._ensure_graph()
                self._graph.replay()
            else:
                self._decode_step()  # first step eager: warms up workspaces before capture
                first = False
            step += 1
            steps_left -= 1
            if steps_left <= 0:
                break
            if step % self.check_every == 0 and self._poll():
                break
        self._check()
        return self.sequences


_ENGINES: "OrderedDict" = OrderedDict()


def _engine_budget(model) -> int:
    """Bytes of KV cache the engine cache may keep alive (``JLA_ENGINE_CACHE_GB`` or 40 % of the device)."""
    env = os.environ.get("JLA_ENGINE_CACHE_GB")
    if env:
        return int(float(env) * (1 << 30))
    if model.device.type == "cuda":
        return int(0.4 * torch.cuda.get_device_properties(model.device).total_memory)
    return 8 << 30


def get_engine(model, batch_size: int, max_length: int) -> DecodeEngine:
    """Per-(model, B, max_length) engines (each owns a KV cache and a captured decode graph), kept in
    LRU order and bounded by the bytes of their KV caches."""
    key = (id(model), batch_size, max_length)
    eng = _ENGINES.get(key)
    if eng is not None:
        _ENGINES.move_to_end(key)
        return eng
    need = model.config.num_hidden_layers * 2 * batch_size * model.n_kv_heads * max_length * model.head_dim * 2
    budget = _engine_budget(model)
    held = sum(e.cache.nbytes() for e in _ENGINES.values())
    while _ENGINES and held + need > budget:
        _, old = _ENGINES.popitem(last=False)
        held -= old.cache.nbytes()
        del old
    eng = DecodeEngine(model, batch_size, max_length)
    _ENGINES[key] = eng
    return eng


def generate(model, input_ids, attention_mask=None, generation_config: Optional[GenerationConfig] = None,
             prng_key=None, **kwargs) -> GenerateOutput:
    # never mutate the caller's config (HF semantics: generate works on a copy)
    gc = dataclasses.replace(generation_config) if generation_config is not None else GenerationConfig()
    for k, v in kwargs.items():
        if hasattr(gc, k):
            setattr(gc, k, v)
    if gc.num_beams != 1:
        raise NotImplementedError("beam search is not used by the reference (num_beams=1)")
    ids = input_ids if torch.is_tensor(input_ids) else torch.as_tensor(input_ids)
    b, s = ids.shape
    if gc.max_length is None:
        gc.max_length = s + (gc.max_new_tokens if gc.max_new_tokens is not None else 20)
    if gc.pad_token_id is None:
        gc.pad_token_id = model.config.pad_token_id if model.config.pad_token_id >= 0 else 0
    if gc.eos_token_id is None:
        gc.eos_token_id = model.config.eos_token_id
    if prng_key is not None:
        gc.seed = int(prng_key) if not torch.is_tensor(prng_key) else int(prng_key.reshape(-1)[0])
    if s >= gc.max_length:
        return GenerateOutput(sequences=ids.to(model.device, torch.int32)[:, : gc.max_length])
    eng = get_engine(model, b, gc.max_length)
    seq = eng.run(ids, attention_mask if attention_mask is None or torch.is_tensor(attention_mask)
                  else torch.as_tensor(attention_mask), gc)
    return GenerateOutput(sequences=seq.clone())
