"""Overlap schedules shared by ``bench.py`` and ``models/``: chunked GEMM on a
(possibly CU-masked) compute stream, collective pieces on the comm stream.

Reference: backup/matmul_overlap_benchmark.py:93-180 (two streams, double
buffer, the collective issued with no dependency on its producer — SURVEY Q7)
and matmul_scaling_benchmark.py:167-238 (matrix_parallel, serialized). Here:

* ``gemm_chunks`` — how many row chunks the GEMM is cut into. A chunk is
  worth having only if its GEMM still fills the chip: with W4 split-K
  (gemm_w4.hip) a chunk of >= 64 256x256 tiles does (S = 4 slices), so the
  8k ws=8 shard (128 tiles) now overlaps in 2 chunks instead of running
  serialized (round 1 required >= 256 tiles per chunk).
* ``GatherOverlap`` — matrix_parallel: GEMM chunk j, then its rows are
  all-gathered in ``pieces`` calls (independent of the GEMM chunking; RCCL's
  all_gather_into_tensor or the direct P2P all-gather, ``impl``),
  each on the comm stream after an event recorded behind chunk j; the step
  ends with the compute stream waiting for every piece (the timed region
  includes the last collective).
* ``ReduceOverlap`` — batch_parallel: (batch element, row chunk) units, each
  all-reduced behind its GEMM.
* ``compute_stream(device, comm_cus)`` — a HIP stream whose kernels may not
  use ``comm_cus`` CUs (hipExtStreamCreateWithCUMask, spread evenly over the
  8 XCDs), so RCCL's workgroups start on those CUs at once instead of waiting
  for a 1-workgroup-per-CU GEMM wave to retire.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from .comm import CommStream, new_event, stream_ctx
from .partition import ceil_div, effective_chunks, row_chunks

# 256x256 output tiles a GEMM chunk needs to fill the chip (ops/gemm.py
# min_chunk_tiles): 64 for the split-K W4 kernel (bf16/fp16), a full wave of
# 256 for the others.
_SPLITK_MIN_TILES = 64


def min_chunk_tiles(dtype: torch.dtype, device: torch.device) -> int:
    if device.type != "cuda":
        return 1
    return _SPLITK_MIN_TILES if dtype in (torch.bfloat16, torch.float16) else 256


def gemm_chunks(m: int, n: int, requested: int, dtype: torch.dtype,
                device: torch.device) -> List[Tuple[int, int]]:
    """Row chunks [start, stop) of an [m, n] GEMM output for an overlap schedule."""
    if device.type != "cuda":
        return row_chunks(m, requested)
    return row_chunks(m, effective_chunks(m, n, requested,
                                          min_tiles=min_chunk_tiles(dtype, device)))


def _xcd_spread(ncu: int, k: int, nxcd: int = 8) -> List[int]:
    """k CU indices spread evenly over the XCDs (HIP CU-mask bit i lands on
    XCD i % nxcd on multi-XCD parts): the first k indices do exactly that."""
    return list(range(min(max(k, 0), ncu)))


class MaskedStream:
    """A CU-masked HIP stream (owned; destroyed with the object). GEMMs issued
    on it should run under ``ops.gemm.cu_budget(self.cus)`` (``budget()``) so
    their grids are planned for the CUs they may use."""

    def __init__(self, device: torch.device, comm_cus: int):
        from ..ops import _native

        self._C = _native.load()
        ncu = torch.cuda.get_device_properties(device).multi_processor_count
        self.excluded = _xcd_spread(ncu, comm_cus)
        self.handle = int(self._C.create_cu_masked_stream(device.index, self.excluded))
        self.stream = torch.cuda.ExternalStream(self.handle, device=device)
        self.device = device
        self.cus = ncu - len(self.excluded)

    def budget(self):
        from ..ops import gemm

        return gemm.cu_budget(self.cus)

    def active_cus(self) -> int:
        mask = self._C.stream_cu_mask(self.handle, self.device.index)
        return sum(bin(int(w) & 0xFFFFFFFF).count("1") for w in mask)

    def close(self) -> None:
        if self.handle:
            torch.cuda.synchronize(self.device)
            self._C.destroy_stream(self.handle)
            self.handle = 0

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def compute_ctx(stream, owner):
    """Context for issuing GEMMs on a compute stream from ``compute_stream``
    while collectives run beside them: the stream, the shared-device flag
    (``ops.gemm.shared_device``: no persistent GEMM kernel that assumes every
    CU is its own), plus the CU budget when the stream is a masked one."""
    import contextlib

    from ..ops import gemm

    st = contextlib.ExitStack()
    st.enter_context(gemm.shared_device())
    if owner is None:
        st.enter_context(stream_ctx(stream))
        return st
    # the masked stream starts behind everything already queued on the
    # caller's stream (operand initialisation, the previous step's join)
    stream.wait_stream(torch.cuda.current_stream(owner.device))
    st.enter_context(stream_ctx(stream))
    st.enter_context(owner.budget())
    return st


def compute_stream(device: torch.device, comm_cus: int = 0):
    """(stream, owner): the current stream (comm_cus == 0) or a CU-masked one."""
    if device.type != "cuda":
        return None, None
    if comm_cus <= 0:
        return torch.cuda.current_stream(device), None
    ms = MaskedStream(device, comm_cus)
    return ms.stream, ms


class GatherOverlap:
    """matrix_parallel overlap: C_local rows in GEMM chunks, each all-gathered in pieces."""

    def __init__(self, n_rows: int, shard: int, ws: int, device: torch.device,
                 out_dtype: torch.dtype, chunks: Sequence[Tuple[int, int]], pieces: int = 0,
                 requested: int = 4, comm: Optional[CommStream] = None, impl: str = "rccl"):
        if impl not in ("rccl", "direct"):
            raise ValueError(f"all-gather impl {impl!r}: rccl | direct")
        self.impl = impl
        self.chunks = list(chunks)
        per = pieces if pieces > 0 else max(1, ceil_div(max(requested, 1), len(self.chunks)))
        self.pieces = []
        for s, e in self.chunks:
            self.pieces.append([(s + ps, s + pe) for ps, pe in row_chunks(e - s, per, align=8)])
        self.bufs = [[torch.empty((ws * (pe - ps), shard), device=device, dtype=out_dtype)
                      for ps, pe in pcs] for pcs in self.pieces]
        self.ready = [new_event(device) for _ in self.chunks]
        self.done = [[new_event(device) for _ in pcs] for pcs in self.pieces]
        self.cs = comm or CommStream(device)
        self.device = device

    @property
    def n_pieces(self) -> int:
        return sum(len(p) for p in self.pieces)

    def step(self, mm, A, B_local, C_local, compute) -> None:
        for j, (s, e) in enumerate(self.chunks):
            mm(A[s:e], B_local, C_local[s:e])
            self.ready[j].record(compute)
            gather = self.cs.all_gather_direct if self.impl == "direct" else self.cs.all_gather_into
            for p, (ps, pe) in enumerate(self.pieces[j]):
                gather(self.bufs[j][p], C_local[ps:pe], after=self.ready[j] if p == 0 else None,
                       done=self.done[j][p])
        if compute is not None:
            for dj in self.done:
                compute.wait_event(dj[-1])  # comm stream is in order: last piece => all

    def gathered(self) -> List[torch.Tensor]:
        """Gather buffers in row order (models.matrix_parallel.assemble)."""
        return [b for bj in self.bufs for b in bj]


class ReduceOverlap:
    """batch_parallel overlap: per (batch element, row chunk) GEMM, then all-reduce."""

    def __init__(self, local_batch: int, chunks: Sequence[Tuple[int, int]],
                 device: torch.device, comm: Optional[CommStream] = None):
        self.units = [(b, s, e) for b in range(local_batch) for (s, e) in chunks]
        self.ready = [new_event(device) for _ in self.units]
        self.done = [new_event(device) for _ in self.units]
        self.cs = comm or CommStream(device)

    def step(self, mm, A, B, C, compute) -> None:
        for u, (b, s, e) in enumerate(self.units):
            mm(A[b, s:e], B[b], C[b, s:e])
            self.ready[u].record(compute)
            self.cs.all_reduce(C[b, s:e], after=self.ready[u], done=self.done[u])
        if compute is not None and self.done:
            compute.wait_event(self.done[-1])


class BidirRing:
    """ring_parallel (models/ring_parallel.py): all-gather-GEMM over both ring
    directions. Rank r's A block (``rp`` rows) is cut into a top and a bottom
    half; tops rotate clockwise (r -> r+1), bottoms counter-clockwise, so each
    hop drives the links to BOTH neighbours. Hop s multiplies the top of rank
    (r - s)'s block and the bottom of rank (r + s)'s block into
    ``C_local[j * rp : (j + 1) * rp]`` while the next halves move."""

    def __init__(self, A_local: torch.Tensor, rp: int, rank: int, ws: int,
                 device: torch.device, comm: Optional[CommStream] = None):
        self.A, self.rp, self.h, self.r, self.ws = A_local, rp, rp // 2, rank, ws
        self.Rt = [torch.empty_like(A_local[:self.h]) for _ in range(2)]
        self.Rb = [torch.empty_like(A_local[self.h:]) for _ in range(2)]
        self.cs = comm or CommStream(device)
        self.gemm_done = [new_event(device) for _ in range(ws)]
        self.recv_done = [new_event(device) for _ in range(max(ws - 1, 0))]
        self.last = None  # event after the most recently issued GEMM (across steps)

    def step(self, mm, B_local, C_local, compute) -> None:
        r, ws, rp, h = self.r, self.ws, self.rp, self.h
        nxt, prv = (r + 1) % ws, (r - 1) % ws
        top, bot = self.A[:h], self.A[h:]
        for s in range(ws):
            if s > 0 and compute is not None:
                compute.wait_event(self.recv_done[s - 1])
            if s < ws - 1:
                # forward both halves, receive the next two while these multiply
                self.cs.exchange_multi([(top, nxt), (bot, prv)],
                                       [(self.Rt[(s + 1) % 2], prv), (self.Rb[(s + 1) % 2], nxt)],
                                       after=self.last, done=self.recv_done[s])
            jt, jb = (r - s) % ws, (r + s) % ws  # whose A rows each half holds
            mm(top, B_local, C_local[jt * rp:jt * rp + h])
            mm(bot, B_local, C_local[jb * rp + h:(jb + 1) * rp])
            self.gemm_done[s].record(compute)
            self.last = self.gemm_done[s]
            if s < ws - 1:
                top, bot = self.Rt[(s + 1) % 2], self.Rb[(s + 1) % 2]


def all_gather_now(out: torch.Tensor, inp: torch.Tensor, impl: str = "rccl",
                   comm: Optional[CommStream] = None) -> None:
    """Serialized all-gather on the current stream: RCCL's
    ``all_gather_into_tensor``, or the direct P2P all-gather (every block over
    its own link) on ``comm`` with the current stream joined behind it."""
    import torch.distributed as dist

    if impl == "rccl":
        dist.all_gather_into_tensor(out, inp)
        return
    dev = inp.device
    cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    ready, done = new_event(dev), new_event(dev)
    ready.record(cur)
    comm.all_gather_direct(out, inp, after=ready, done=done)
    if cur is not None:
        cur.wait_event(done)
