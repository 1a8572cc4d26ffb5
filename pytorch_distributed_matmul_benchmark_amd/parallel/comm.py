"""Communication streams with explicit event ordering (compute ∥ RCCL).

The reference's overlap variants (backup/matmul_overlap_benchmark.py:93-278)
put collectives on a side stream with no dependency on the GEMM that
produced the buffer and drop the async handle, so the all-reduce can read a
half-written C and the next GEMM can overwrite a buffer that is still being
reduced. Here every hand-off is an event:

    compute: GEMM(buf) → record(ready[buf])
    comm:    wait(ready[buf]) → RCCL collective(buf) → record(done[buf])
    compute: wait(done[buf]) before the next GEMM writes buf

``CommStream.collective`` issues the RCCL op while the comm stream is
current, so ProcessGroupNCCL orders its internal stream after the comm
stream's prior work (the ready-event wait), and ``work.wait()`` makes the
comm stream (not the host) wait for the collective, so ``done`` really
means "reduced". On MI355X the comm stream is created with the highest
priority so RCCL's workgroups are dispatched ahead of queued GEMM
workgroups as CUs free up (the GEMM grid is ≫256 WGs at 1 WG/CU).

On CPU tensors (gloo) streams/events are no-ops and collectives are
synchronous, which keeps the same code path testable without a GPU.
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.distributed as dist


class _NullEvent:
    def record(self, stream=None):
        pass

    def wait(self, stream=None):
        pass

    def synchronize(self):
        pass

    def elapsed_time(self, other):
        return 0.0


def new_event(device: torch.device, timing: bool = False):
    if device.type == "cuda":
        return torch.cuda.Event(enable_timing=timing)
    return _NullEvent()


def new_stream(device: torch.device, high_priority: bool = False):
    if device.type != "cuda":
        return None
    if high_priority:
        lo, hi = torch.cuda.Stream.priority_range()
        return torch.cuda.Stream(device=device, priority=hi)
    return torch.cuda.Stream(device=device)


def stream_ctx(stream):
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def current_stream(device: torch.device):
    return torch.cuda.current_stream(device) if device.type == "cuda" else None


class CommStream:
    """A dedicated stream for RCCL collectives, ordered by events against compute."""

    def __init__(self, device: torch.device, group=None, high_priority: bool = True):
        self.device = device
        self.group = group
        self.stream = new_stream(device, high_priority=high_priority)

    def wait_event(self, ev) -> None:
        if self.stream is not None and ev is not None:
            self.stream.wait_event(ev)

    def collective(self, fn, *args, after=None, done=None, **kw):
        """Run ``fn(*args, async_op=True, **kw)`` on the comm stream.

        ``after``: event the collective must wait for (the producer GEMM).
        ``done``: event recorded once the collective has completed on the GPU.
        """
        with stream_ctx(self.stream):
            if after is not None:
                self.wait_event(after)
            work = fn(*args, group=self.group, async_op=True, **kw)
            if work is not None:
                work.wait()  # NCCL: stream-side wait only; gloo: blocks (CPU)
            if done is not None:
                done.record(self.stream)
        return work

    def all_reduce(self, t: torch.Tensor, after=None, done=None):
        return self.collective(dist.all_reduce, t, after=after, done=done)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, after=None, done=None):
        return self.collective(dist.all_gather_into_tensor, out, inp, after=after, done=done)

    def exchange(self, send: torch.Tensor, dst: int, recv: torch.Tensor, src: int,
                 after=None, done=None):
        """One ring hop on the comm stream: ``send`` → rank ``dst`` while ``recv``
        ← rank ``src`` (global ranks), issued as one batched P2P group so RCCL
        runs both directions of the hop concurrently."""
        return self.exchange_multi([(send, dst)], [(recv, src)], after=after, done=done)

    def exchange_multi(self, sends, recvs, after=None, done=None):
        """Several point-to-point transfers as ONE batched group on the comm
        stream (``sends``: [(tensor, dst)], ``recvs``: [(tensor, src)]). The
        bidirectional ring sends half a block to each neighbour this way, so
        every hop drives two xGMI links (one per direction) instead of one.
        Transfer i carries tag i (gloo matches on it; RCCL matches in issue
        order, which is the same list order on every rank), so two transfers
        between the same pair (ws = 2) never cross; a (tensor, rank, tag)
        triple sets the tag explicitly (lists that skip empty transfers)."""
        with stream_ctx(self.stream):
            if after is not None:
                self.wait_event(after)
            # gloo P2P takes host memory only: GPU tensors of a gloo rehearsal
            # (ranks sharing one GPU) hop through host copies on this stream.
            first = (list(sends) + list(recvs))[:1]
            staged = bool(first) and first[0][0].is_cuda and dist.get_backend(self.group) == "gloo"
            ops, landing = [], []
            for i in range(max(len(sends), len(recvs))):
                if i < len(sends):
                    t, dst, *tag = sends[i]
                    ops.append(dist.P2POp(dist.isend, t.cpu() if staged else t, dst,
                                          group=self.group, tag=tag[0] if tag else i))
                if i < len(recvs):
                    t, src, *tag = recvs[i]
                    r_t = torch.empty(t.shape, dtype=t.dtype) if staged else t
                    landing.append((t, r_t))
                    ops.append(dist.P2POp(dist.irecv, r_t, src, group=self.group,
                                          tag=tag[0] if tag else i))
            if not ops:
                if done is not None:
                    done.record(self.stream)
                return []
            works = dist.batch_isend_irecv(ops)
            for wk in works:
                wk.wait()
            if staged:
                for t, r_t in landing:
                    t.copy_(r_t)
            if done is not None:
                done.record(self.stream)
        return works

    def all_gather_direct(self, out: torch.Tensor, inp: torch.Tensor, after=None, done=None):
        """All-gather as ONE batched group of point-to-point transfers: this
        rank's ``inp`` goes straight to every other rank and every other
        rank's block lands straight in its slot of ``out`` ([ws * rows, ...],
        block r = rank r's ``inp``). On a fully connected 8 x MI355X node each
        of the ws-1 transfers has its own xGMI link, so all 7 links carry
        data at once with no forwarding hop (RCCL's ring all-gather forwards
        every block ws-1 times). Selected with ``--allgather direct``."""
        group_ws = dist.get_world_size(self.group)
        me = dist.get_rank(self.group)
        rows = inp.shape[0]
        blocks = [out[r * rows:(r + 1) * rows] for r in range(group_ws)]
        with stream_ctx(self.stream):
            if after is not None:
                self.wait_event(after)
            blocks[me].copy_(inp)
        peers = [(me + d) % group_ws for d in range(1, group_ws)]
        g = lambda r: dist.get_global_rank(self.group, r) if self.group is not None else r  # noqa: E731
        return self.exchange_multi([(inp, g(p)) for p in peers],
                                   [(blocks[(me - d) % group_ws], g((me - d) % group_ws))
                                    for d in range(1, group_ws)],
                                   after=None, done=done)

    def _scratch(self, t: torch.Tensor, numel: int) -> torch.Tensor:
        """Landing space for the ws-1 chunks of the reduce-scatter phase, one
        per (device, dtype), grown on demand. Only the comm stream touches it,
        so stream order makes reuse across collectives safe."""
        buf = getattr(self, "_ar_scratch", None)
        if buf is None or buf.dtype != t.dtype or buf.numel() < numel:
            with stream_ctx(self.stream):
                buf = torch.empty(max(numel, 1), dtype=t.dtype, device=t.device)
            self._ar_scratch = buf
        return buf

    def all_reduce_direct(self, t: torch.Tensor, after=None, done=None):
        """SUM all-reduce of contiguous ``t`` as a two-shot exchange over
        point-to-point links (``--allreduce direct``):

          1. reduce-scatter: ``t`` is cut into ws chunks (64-element multiples);
             chunk p goes straight to rank p and every peer's copy of this
             rank's chunk lands in a scratch slot, as ONE batched P2P group;
          2. the native ``reduce_sum`` kernel (ops/csrc/reduce.hip) adds the ws
             copies in rank order with fp32 accumulation into this rank's chunk;
          3. all-gather: the reduced chunk goes to every peer, theirs land in
             place, again one batched group.

        On a fully connected 8 x MI355X node every transfer of a phase has its
        own xGMI link, each byte crosses a link twice (RCCL's ring all-reduce:
        2(ws-1)/ws of the buffer through every ring hop), and the sum is exact
        to fp32 then rounded once (a ring rounds after every hop). Ranks sum in
        the same order, so every rank gets identical bits."""
        assert t.is_contiguous(), "all_reduce_direct needs a contiguous tensor"
        group_ws = dist.get_world_size(self.group)
        me = dist.get_rank(self.group)
        flat = t.view(-1)
        n = flat.numel()
        if group_ws == 1 or n == 0:
            with stream_ctx(self.stream):
                if after is not None:
                    self.wait_event(after)
                if done is not None:
                    done.record(self.stream)
            return None
        chunk = -(-n // group_ws)
        chunk = -(-chunk // 64) * 64  # 16-B aligned chunk starts for every dtype
        bounds = [(min(r * chunk, n), min((r + 1) * chunk, n)) for r in range(group_ws)]
        part = [flat[s:e] for s, e in bounds]
        mine = part[me]
        m = mine.numel()
        g = lambda r: dist.get_global_rank(self.group, r) if self.group is not None else r  # noqa: E731
        peers = [(me + d) % group_ws for d in range(1, group_ws)]
        srcs = [(me - d) % group_ws for d in range(1, group_ws)]
        scratch = self._scratch(t, (group_ws - 1) * chunk)
        slot = {src: scratch[i * chunk:i * chunk + m] for i, src in enumerate(srcs)}
        # 1. reduce-scatter (chunks past the end are empty on every rank alike;
        # the tag is the ring distance d, the same at both ends of a transfer)
        sends = [(part[p], g(p), d) for d, p in enumerate(peers, 1) if part[p].numel()]
        recvs = [(slot[s], g(s), d) for d, s in enumerate(srcs, 1) if m]
        self.exchange_multi(sends, recvs, after=after)
        # 2. local sum in rank order
        with stream_ctx(self.stream):
            if m:
                ordered = [mine if r == me else slot[r] for r in range(group_ws)]
                reduce_sum_(mine, ordered)
        # 3. all-gather of the reduced chunks
        sends = [(mine, g(p), d) for d, p in enumerate(peers, 1)] if m else []
        recvs = [(part[s], g(s), d) for d, s in enumerate(srcs, 1) if part[s].numel()]
        return self.exchange_multi(sends, recvs, done=done)

    def synchronize(self) -> None:
        if self.stream is not None:
            self.stream.synchronize()


def reduce_sum_(out: torch.Tensor, srcs) -> None:
    """out = sum(srcs) with fp32 accumulation in list order, rounded once (out
    may be one of srcs). GPU tensors run the native ``reduce_sum`` kernel —
    no eager fallback on a GPU; CPU tensors (gloo rehearsals) the same sum in
    torch."""
    if out.is_cuda:
        from ..ops import _native

        _native.load(build_if_missing=False).reduce_sum(out, list(srcs))
        return
    acc = torch.zeros(out.shape, dtype=torch.float32)
    for s in srcs:
        acc += s.float()
    out.copy_(acc)


def all_reduce_(t: torch.Tensor, group=None) -> None:
    """Synchronous (stream-ordered) in-place SUM all-reduce on the current stream."""
    dist.all_reduce(t, group=group)


def all_gather_into_(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    dist.all_gather_into_tensor(out, inp, group=group)

