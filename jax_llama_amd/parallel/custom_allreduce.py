"""Custom xGMI collectives for decode-sized tensor-parallel messages (``csrc/kernels/allreduce.hip``).

SURVEY D1: RCCL (``torch.distributed`` backend ``nccl``) carries init, large (prefill) messages and is
the correctness oracle. The per-token collectives of the decode step go through these kernels instead,
so a captured decode step contains no RCCL call at all:

  * ``all_reduce_residual_(partial, h, hb)`` — the 2 row-parallel sums per layer (reference
    ``partition.py:67,70``: XLA inserts them after ``wo`` and ``w2``) with the residual add and the
    bf16 mirror of the residual stream fused into the reduction (``h += sum``, ``hb = bf16(h)``);
  * ``argmax_pairs(val, idx, offset)`` — vocab-parallel greedy token (``partition.py:77``): every
    rank's (max, argmax) is all-gathered and reduced to the first max in rank order;
  * ``topk_pairs(vals, idx, offset)`` — every rank's top-k candidates, gathered as ``[B, tp*k]``
    for the exact distributed sampler.

One-shot (every rank reads every peer's copy) for small messages; two-shot (reduce-scatter +
all-gather of the fp32 sums) for large ones at >= 4 ranks, where it moves ``3/world`` of the bytes
per link. Both sum in rank order in fp32, so they are bit-identical to each other and on every rank.

Rendezvous: each rank allocates its buffers, the IPC handles are exchanged with
``all_gather_object`` on the TP group, then every rank maps its peers'. A peer that never arrives
makes the kernel give up after ``timeout_s`` and set an error word (every later wait then gives up at
once, so nothing hangs); ``check()`` raises on it and the object refuses every later call.
"""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist

from ..ops import ext

# Two-shot above this many bytes per rank (at >= 4 ranks). One-shot moves (world-1) x bytes per rank over
# world-1 links (bytes per link); two-shot moves 3 x bytes / world per link (bf16 partial scatter + fp32 sum
# gather) at the price of a second barrier.
TWO_SHOT_MIN_BYTES = int(os.environ.get("JLA_CAR_TWO_SHOT_BYTES", str(512 << 10)))
CHUNK_BYTES = 4096  # allreduce.hip CAR_CHUNK: buffers hold whole chunks


class CustomAllReduceError(RuntimeError):
    pass


class CustomAllReduce:
    DTYPES = (torch.bfloat16, torch.float32)

    def __init__(self, state: int, rank: int, world: int, max_bytes: int, share: int = 1, group=None):
        self.state = state
        self.rank = rank
        self.world = world
        self.size = world  # (autotune.tp_scope reads size / rank / group)
        self.group = group
        self.max_bytes = max_bytes
        # most ranks of the group on one device (1 on a real node; > 1 when test ranks share a GPU): the fused GEMV's
        # workgroups spin for their peers', so every rank's grid must fit on a shared device at once
        self.share = share
        self.failed = False  # set once a timeout was seen: the per-block counters are out of step for good
        self.litmus = None  # verdict of self_test (create_for runs it)

    def _live(self) -> int:
        if self.failed:
            raise CustomAllReduceError("custom all-reduce timed out earlier; re-create it (every rank) before reuse")
        if not self.state:
            raise CustomAllReduceError("custom all-reduce is closed")
        return self.state

    @classmethod
    def create(cls, ctx, max_bytes: int = 16 << 20, group=None, timeout_s: float = 10.0,
               kind: str = "collective") -> "CustomAllReduce":
        return cls.create_for(ctx.tp_rank, ctx.tp_size, ctx.tp_group if group is None else group, max_bytes,
                              timeout_s, kind)

    @classmethod
    def create_for(cls, rank: int, world: int, group, max_bytes: int = 16 << 20,
                   timeout_s: float = 10.0, kind: str = "collective") -> "CustomAllReduce":
        """``kind``: which litmus ``self_test`` runs before the instance is handed out (``collective``: the
        standalone all-reduce / gather paths; ``fused``: the GEMV-fused row-parallel exchange)."""
        if world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI hop)")
        max_bytes = (max_bytes + CHUNK_BYTES - 1) // CHUNK_BYTES * CHUNK_BYTES  # whole kernel chunks
        e = ext()
        buf = sig = 0
        state, err = 0, None
        try:
            buf, sig, hbuf, hsig = e.car_alloc(max_bytes, world)
            mine = (bytes(hbuf), bytes(hsig))
        except RuntimeError as ex:  # allocation / IPC export failed here: still join the rendezvous
            mine, err = None, f"car_alloc: {ex}"
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        if err is None and all(h is not None for h in handles):
            try:
                state = e.car_init(rank, world, max_bytes, buf, sig, [h[0] for h in handles], [h[1] for h in handles],
                                   float(timeout_s))
            except RuntimeError as ex:  # e.g. the IPC import failed on this rank
                state, err = 0, str(ex)
        elif err is None:
            err = "a peer failed to allocate its buffers"
        # every rank learns whether every rank mapped its peers: one rank failing must not leave the
        # others spinning in a collective it will never join -- and none may keep its mappings or buffers
        oks = [None] * world
        dist.all_gather_object(oks, err is None, group=group)
        if not all(oks):
            if state:
                e.car_destroy(state)  # unmaps the peers and frees this rank's buffers
            else:
                e.car_free(buf, sig)
            raise CustomAllReduceError(f"custom all-reduce setup failed on ranks "
                                       f"{[r for r, ok in enumerate(oks) if not ok]}: {err}")
        dev = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(dev)
        key = (socket.gethostname(), p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        keys = [None] * world
        dist.all_gather_object(keys, key, group=group)
        car = cls(state, rank, world, max_bytes, share=max(keys.count(k) for k in keys), group=group)
        grid = int(os.environ.get("JLA_CAR_GRID", "0"))  # tests: pin the grid (the same on every rank)
        if grid > 0:
            e.car_set_grid(state, grid)
        elif car.share == 1:
            # one rank per GPU: up to 255 collective blocks (a 4 MiB partial over every CU); ranks sharing a device
            # keep 63 so every rank's blocks stay co-resident (they spin for each other). Same value on every rank,
            # set before the first call (the self-test): the chunk -> block map must never change under an instance.
            e.car_set_grid(state, 0)
        # protocol litmus on the real links: every path, rank-dependent data, every word checked on the host
        try:
            ok = car.self_test(kind)
        except Exception as ex:  # noqa: BLE001 -- a failing path is a failed litmus, on every rank
            import logging
            logging.getLogger(__name__).warning("custom all-reduce litmus raised: %s", ex)
            ok = False
        dist.all_gather_object(oks, ok, group=group)
        if not all(oks):
            car.close()
            raise CustomAllReduceError("custom all-reduce self-test failed (wrong sums or a timeout)")
        return car

    @classmethod
    def local(cls, max_bytes: int = 16 << 20, timeout_s: float = 10.0) -> "CustomAllReduce":
        """A world-1 instance (no rendezvous): the same kernels, launch structure and hand-off protocol with this
        rank as its only peer -- the collective of the one-GPU tensor-parallel rank proxy (``TPRankProxyComm``)."""
        max_bytes = (max_bytes + CHUNK_BYTES - 1) // CHUNK_BYTES * CHUNK_BYTES
        e = ext()
        buf, sig, hbuf, hsig = e.car_alloc(max_bytes, 1)
        try:
            state = e.car_init(0, 1, max_bytes, buf, sig, [bytes(hbuf)], [bytes(hsig)], float(timeout_s))
        except RuntimeError:
            e.car_free(buf, sig)
            raise
        # the only rank on its GPU: the full collective grid, as a TP rank on its own GPU (JLA_CAR_GRID pins one: A/B)
        e.car_set_grid(state, int(os.environ.get("JLA_CAR_GRID", "0")))
        return cls(state, 0, 1, max_bytes)

    LITMUS_ROUNDS = int(os.environ.get("JLA_CAR_LITMUS_ROUNDS", "8"))

    @staticmethod
    def _pattern(n: int, rank: int, rnd: int) -> torch.Tensor:
        """Rank- and round-dependent integers in [1, 97]: exact in bf16 and fp32, and so are their sums over <= 8
        ranks -- every rank can compute every peer's data and the exact expected result on the host."""
        return ((torch.arange(n, dtype=torch.int64) * (2 * rnd + 1) + 31 * rank + rnd) % 97 + 1).to(torch.float32)

    def self_test(self, kind: str = "collective", rounds=None) -> bool:
        """Litmus test on the real links before the instance is declared usable (a wrong protocol on some fabric
        must fall back to RCCL, not corrupt a generation): ``rounds`` rounds of every path with rank- and
        round-dependent data, every word checked exactly on the host. ``collective``: granule one-shot (fp32 sum
        and the bf16 residual epilogue), flag one-shot (> the granule limit), two-shot, and the (value, index) pair
        gather; ``fused``: the GEMV-fused row-parallel exchange (gemv.hip MODE_TPRESID) and the tiled GEMM's fused reduce
        (gemm.hip gemm_reduce_tp_kernel). The verdict and the paths
        checked are kept in ``self.litmus``."""
        rounds = self.LITMUS_ROUNDS if rounds is None else rounds
        world, rank = self.world, self.rank
        paths = []
        ok = True

        def want_sum(n, rnd):
            return sum(self._pattern(n, r, rnd) for r in range(world))

        for rnd in range(rounds):
            if kind == "fused":
                from ..models.weights import PackedLinear
                m, n, k = 4, 256, 256
                if not self.can_fuse(m, n):
                    break
                # W_rank[n][k] = 1 where (n + k + rank) % 3 == rnd % 3: every partial is an exact bf16 integer
                def wmat(r):
                    nn = torch.arange(n)[:, None]
                    kk = torch.arange(k)[None, :]
                    return ((nn + kk + r) % 3 == rnd % 3).to(torch.bfloat16)
                w = PackedLinear.from_dense(wmat(rank), "cuda")
                x = torch.ones(m, k, dtype=torch.bfloat16, device="cuda")
                h = (torch.arange(m * n, dtype=torch.float32) % 13).reshape(m, n).cuda()
                hb = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
                want = (torch.arange(m * n, dtype=torch.float32) % 13).reshape(m, n) + sum(
                    wmat(r).float().sum(1) for r in range(world))[None, :]
                self.linear_residual_(x, w, h, hb)
                ok = ok and torch.equal(h.cpu(), want) and torch.equal(hb.cpu(), want.to(torch.bfloat16))
                paths = ["fused_gemv"]
                # the tiled GEMM's split-K reduce with the exchange (gemm.hip gemm_reduce_tp_kernel: 16-byte gathers)
                mt = 96
                if self.can_fuse_tiled(mt, n):
                    from .. import ops
                    xt = torch.ones(mt, k, dtype=torch.bfloat16, device="cuda")
                    ht = (torch.arange(mt * n, dtype=torch.float32) % 13).reshape(mt, n).cuda()
                    hbt = torch.empty(mt, n, dtype=torch.bfloat16, device="cuda")
                    ws = torch.empty(2 * mt * (n + 1), dtype=torch.float32, device="cuda")
                    ops.ext().gemm_tp_residual(self._live(), xt, w.weight, n, k, ht, hbt, 2, ws, 1)
                    wt = (torch.arange(mt * n, dtype=torch.float32) % 13).reshape(mt, n) + sum(
                        wmat(r).float().sum(1) for r in range(world))[None, :]
                    ok = ok and torch.equal(ht.cpu(), wt) and torch.equal(hbt.cpu(), wt.to(torch.bfloat16))
                    paths = ["fused_gemv", "fused_tiled_reduce"]
                continue
            # granule one-shot (fp32 sum), flag one-shot (fp32, above the granule limit), two-shot (forced)
            for name, n, ts in (("granule", 16 * 1024, False), ("flag", 192 * 1024, False), ("two_shot", 64 * 1024, True)):
                if n * 4 > self.max_bytes:
                    continue
                got = self.all_reduce(self._pattern(n, rank, rnd).cuda(), two_shot=ts).cpu()
                ok = ok and torch.equal(got, want_sum(n, rnd))
                if rnd == 0:
                    paths.append(name)
            # the residual epilogue with bf16 partials, on the granule and on the flag path
            for name, n in (("granule_resid_bf16", 8 * 1024), ("flag_resid_bf16", 256 * 1024)):
                if n * 2 > self.max_bytes:
                    continue
                h0 = (torch.arange(n, dtype=torch.float32) % 13)
                h = h0.cuda()
                hb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
                self.all_reduce_residual_(self._pattern(n, rank, rnd).to(torch.bfloat16).cuda(), h, hb)
                want = h0 + want_sum(n, rnd)
                ok = ok and torch.equal(h.cpu(), want) and torch.equal(hb.cpu(), want.to(torch.bfloat16))
                if rnd == 0:
                    paths.append(name)
            # (value, index) pairs: the first max over ranks, rank order breaking ties
            b = 256
            vals = [((torch.arange(b) * 7 + 3 * r + rnd) % 11).to(torch.float32) for r in range(world)]
            got = self.argmax_pairs(vals[rank].cuda(), torch.arange(b, dtype=torch.int32, device="cuda"),
                                    rank * b).cpu()
            stacked = torch.stack(vals)  # [world, b]
            best = stacked.argmax(0)  # first max in rank order
            ok = ok and torch.equal(got, (best * b + torch.arange(b)).to(torch.int32))
            if rnd == 0:
                paths.append("pairs")
        torch.cuda.synchronize()
        ok = bool(ok and self.error() == 0)
        self.litmus = {"kind": kind, "rounds": rounds, "paths": paths, "ok": ok}
        return ok

    # ------------------------------------------------------------------ capability checks
    def can_handle(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and t.dtype in self.DTYPES and 0 < nbytes <= self.max_bytes
                and nbytes % 16 == 0)

    def can_handle_pairs(self, n: int) -> bool:
        return 0 < n * 8 <= self.max_bytes

    def use_two_shot(self, nbytes: int) -> bool:
        return self.world >= 4 and nbytes >= TWO_SHOT_MIN_BYTES

    # ------------------------------------------------------------------ collectives
    def all_reduce_(self, t: torch.Tensor, two_shot=None) -> torch.Tensor:
        ts = self.use_two_shot(t.numel() * t.element_size()) if two_shot is None else bool(two_shot)
        ext().car_allreduce(self._live(), t, t, ts)
        return t

    def all_reduce(self, t: torch.Tensor, two_shot=None) -> torch.Tensor:
        out = torch.empty_like(t)
        ts = self.use_two_shot(t.numel() * t.element_size()) if two_shot is None else bool(two_shot)
        ext().car_allreduce(self._live(), t, out, ts)
        return out

    def all_reduce_residual_(self, partial: torch.Tensor, h: torch.Tensor, hb: torch.Tensor, two_shot=None,
                             hb_pack=None):
        """``h += sum_ranks(partial)``; ``hb = bf16(h)`` (one kernel); ``hb_pack``: also a packed-layout copy of hb
        (``ops.packed_rows`` x D, the next projection's packed-x input)."""
        ts = self.use_two_shot(partial.numel() * partial.element_size()) if two_shot is None else bool(two_shot)
        ext().car_allreduce_residual(self._live(), partial, h, hb, ts, hb_pack)

    # fused row-parallel GEMV (gemv.hip MODE_TPRESID): one TPRES_REGION of the slot per workgroup (<= 1 per 16
    # output columns), at most WG_COUNTERS workgroups
    TPRES_REGION = 64 * 64 * 4
    WG_COUNTERS = 4096

    SHARED_MAX_GROUPS = 256  # ranks sharing a device: all their workgroups resident at once (<= 16 waves, 64 KiB LDS)

    def can_fuse(self, m: int, n: int) -> bool:
        groups = n // 16
        return (1 <= m <= 64 and n % 16 == 0 and groups <= self.WG_COUNTERS and groups * self.TPRES_REGION <=
                self.max_bytes and (self.share == 1 or self.share * groups <= self.SHARED_MAX_GROUPS))

    def linear_residual_(self, x: torch.Tensor, w, h: torch.Tensor, hb: torch.Tensor, x_packed=None, hb_pack=None):
        """``h += sum_ranks(x @ W^T)``, ``hb = bf16(h)``: the GEMV exchanges its bf16 partials itself (no separate
        collective). Uses this instance's per-workgroup counters: reserve an instance for it. Every rank must launch
        the same GEMV variant (workgroup w of every rank covers the same columns): rank 0 picks it."""
        from .. import ops
        with ops.autotune.tp_scope(self):
            ops.linear_tp_residual(x, w, h, hb, self._live(), x_packed=x_packed, hb_pack=hb_pack)

    def can_fuse_tiled(self, m: int, n: int) -> bool:
        """The tiled GEMM's fused path (decode batches past the GEMV's rows): one region + counter per 4096 output
        elements (csrc/kernels/gemm.hip gemm_reduce_tp_kernel)."""
        groups = (m * n + 4095) // 4096
        return (m > 0 and n % 4 == 0 and groups <= self.WG_COUNTERS and groups * self.TPRES_REGION <= self.max_bytes
                and (self.share == 1 or self.share * groups <= self.SHARED_MAX_GROUPS))

    def tiled_residual_(self, x: torch.Tensor, w, h: torch.Tensor, hb: torch.Tensor) -> bool:
        """``h += sum_ranks(x @ W^T)``, ``hb = bf16(h)`` with the exchange in the split-K reduce of the tiled GEMM.
        False (nothing done) when the tuned plan for this shape has no K split. Rank 0 picks the plan."""
        from .. import ops
        with ops.autotune.tp_scope(self):
            return ops.tiled_tp_residual(x, w, h, hb, self._live())

    @staticmethod
    def fused_bytes(hidden: int) -> int:
        """Slot bytes the fused path needs for a row-parallel output of ``hidden`` columns."""
        return max(CHUNK_BYTES, (hidden // 16) * CustomAllReduce.TPRES_REGION)

    def argmax_pairs(self, val: torch.Tensor, idx: torch.Tensor, idx_offset: int, out_val=None) -> torch.Tensor:
        """First max over ranks of each row's local ``(val, idx + idx_offset)``: int32 ``[B]``."""
        out = torch.empty(idx.numel(), dtype=torch.int32, device=idx.device)
        ext().car_pairs(self._live(), 0, val.contiguous(), idx.contiguous(), int(idx_offset), 1, out_val, out)
        return out

    def topk_pairs(self, vals: torch.Tensor, idx: torch.Tensor, idx_offset: int):
        """``[B, k]`` local candidates of every rank -> ``(vals, idx)`` of shape ``[B, world * k]``."""
        b, k = vals.shape
        ov = torch.empty(b, self.world * k, dtype=torch.float32, device=vals.device)
        oi = torch.empty(b, self.world * k, dtype=torch.int32, device=vals.device)
        ext().car_pairs(self._live(), 1, vals.contiguous(), idx.contiguous(), int(idx_offset), int(k), ov, oi)
        return ov, oi

    # ------------------------------------------------------------------ failure detection
    def error(self) -> int:
        """1 if a kernel gave up waiting for a peer (bounded spin) since creation."""
        return int(ext().car_error(self.state))

    def check(self):
        """Raise if a kernel gave up waiting (the host's periodic poll). From then on every call raises too:
        the per-block call / barrier counters are out of step with the peers', so the object must be
        re-created on every rank."""
        if self.failed or (self.state and self.error()):
            self.failed = True
            raise CustomAllReduceError(
                "custom all-reduce: a peer did not arrive within the timeout; results since then are invalid")

    def close(self):
        if self.state:
            ext().car_destroy(self.state)
            self.state = 0
