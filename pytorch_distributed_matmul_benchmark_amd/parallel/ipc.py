"""Collectives over xGMI peer memory (``--allgather ipc``, ``--allreduce ipc``).

All-gather: every rank PULLS each
peer's shard straight out of that peer's memory with DMA-engine copies, one
copy stream per peer, so on a fully connected 8 x MI355X node the seven
transfers run over seven xGMI links at once and use no CUs — the GEMM the
collective overlaps keeps every CU (an RCCL all-gather runs its channels as
kernels on the same CUs).

SURVEY §7.2 (K5-K7 stretch): "custom xGMI peer-memory all-gather (hipIpc
handles, 7 links in parallel)"; the reference's all-gather call site is
matmul_scaling_benchmark.py:204-224 (NCCL ``all_gather``).

Mechanics (ops/csrc/bindings.cpp ``ipc_*`` / ``copy_from_peer``):

  * ``register(src)``: ``src`` (an ``ipc_empty`` tensor: its own hipMalloc
    allocation) is exported with ``hipIpcGetMemHandle``; the handles are
    exchanged once (a host all-gather of objects) and every peer's is mapped
    with ``hipIpcOpenMemHandle``. Every rank registers corresponding buffers
    in the same order.
  * ``all_gather(out, inp, after, done)``: ``inp`` is a view into a
    registered buffer (the same offset on every rank, e.g. a row block of
    the local output C). On the comm stream: wait ``after``; copy the local
    block; fork one copy stream per peer and ``hipMemcpyAsync`` that peer's
    block (same offset in ITS buffer) into ``out``; join; then a
    stream-ordered barrier (a one-element RCCL all-reduce): when it
    completes on a rank, every peer has finished pulling from that rank, so
    the rank's next GEMM may overwrite its shard (pull keeps ``out`` written
    only by its owner, so no cross-rank hazard on the gathered buffer);
    record ``done``.
  * ``close()``: unmap the peers' buffers, then a barrier, so no rank frees
    an exported buffer another rank still maps.

``all_reduce(t)`` is the direct two-shot all-reduce on the same mappings:
pull this rank's chunk from every peer, ``reduce_sum`` in rank order, pull
every peer's reduced chunk, with three stream-ordered barriers (method
docstring).

gloo rehearsals (ranks sharing one GPU) exchange handles the same way; the
barrier becomes a host barrier after the comm stream drains. CPU tensors have
no peer memory: ``--allgather ipc`` falls back to the direct P2P all-gather
there (parallel/comm.py ``all_gather_direct``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .comm import CommStream, stream_ctx


def _mod():
    from ..ops import _native

    return _native.load(build_if_missing=False)


def ipc_empty(shape, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """A GPU tensor in its own allocation (IPC-exportable); CPU: plain empty."""
    if device.type != "cuda":
        return torch.empty(shape, dtype=dtype, device=device)
    return _mod().ipc_empty(list(shape), dtype, device.index if device.index is not None else 0)


class IpcGather:
    """Peer-memory all-gather on a CommStream (module docstring)."""

    def __init__(self, comm: CommStream, group=None):
        self.cs = comm
        self.group = group
        self.device = comm.device
        self.ws = dist.get_world_size(group)
        self.me = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        # registered buffers: (local base address, bytes) -> {peer rank: mapped address}
        self.bufs: List[Tuple[int, int, Dict[int, int]]] = []
        self.copy_streams = [torch.cuda.Stream(device=self.device) for _ in range(max(self.ws - 1, 0))]
        self.flag = torch.zeros(1, device=self.device)

    def register(self, src: torch.Tensor) -> None:
        """Export ``src`` and map every peer's corresponding buffer (collective)."""
        assert src.is_cuda and src.storage_offset() == 0, "register an ipc_empty tensor"
        mod = _mod()
        mine = mod.ipc_handle(src)
        handles: List[Optional[bytes]] = [None] * self.ws
        dist.all_gather_object(handles, mine, group=self.group)
        peers = {r: mod.ipc_open(h, self.dev_index) for r, h in enumerate(handles) if r != self.me}
        self.bufs.append((src.data_ptr(), src.untyped_storage().nbytes(), peers))

    def _peer_addr(self, t: torch.Tensor, peer: int) -> int:
        p = t.data_ptr()
        for base, nbytes, peers in self.bufs:
            if base <= p and p + t.nbytes <= base + nbytes:
                return peers[peer] + (p - base)
        raise ValueError("IpcGather: the input is not inside a registered buffer")

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, after=None, done=None) -> None:
        """``out`` [ws * rows, ...] (contiguous) <- every rank's ``inp`` [rows, ...]."""
        assert inp.is_contiguous() and out.is_contiguous()
        rows = inp.shape[0]
        blocks = [out[r * rows:(r + 1) * rows] for r in range(self.ws)]
        mod = _mod()
        cs = self.cs.stream
        with stream_ctx(cs):
            if after is not None:
                cs.wait_event(after)
            blocks[self.me].copy_(inp)
            fork = torch.cuda.Event()
            fork.record(cs)
        joins = []
        for i, d in enumerate(range(1, self.ws)):
            p = (self.me + d) % self.ws
            st = self.copy_streams[i]
            with torch.cuda.stream(st):
                st.wait_event(fork)
                mod.copy_from_peer(blocks[p], self._peer_addr(inp, p))
                ev = torch.cuda.Event()
                ev.record(st)
                joins.append(ev)
        with stream_ctx(cs):
            for ev in joins:
                cs.wait_event(ev)
            self._barrier()
            if done is not None:
                done.record(cs)

    def all_reduce(self, t: torch.Tensor, after=None, done=None) -> None:
        """SUM all-reduce of ``t`` (a contiguous view into a registered buffer,
        the same offsets on every rank) over peer memory — the direct
        two-shot exchange of ``CommStream.all_reduce_direct`` with pulls
        instead of P2P sends, so DMA engines move the bytes and no CUs do:

          B0 barrier (every rank's ``t`` final) -> pull chunk ``me`` of every
          peer's ``t`` into scratch (one copy stream per peer) -> native
          ``reduce_sum`` in rank order into this rank's chunk -> B1 barrier
          (every chunk reduced) -> pull every peer's reduced chunk into place
          -> B2 barrier (no peer still reads this rank's chunk when its next
          producer overwrites ``t``).

        Chunks are 64-element multiples (16-B aligned); every rank sums in the
        same order, so all ranks hold identical bits."""
        from .comm import reduce_sum_

        assert t.is_contiguous()
        if self.ws == 1 or t.numel() == 0:
            with stream_ctx(self.cs.stream):
                if after is not None:
                    self.cs.stream.wait_event(after)
                if done is not None:
                    done.record(self.cs.stream)
            return
        mod = _mod()
        cs = self.cs.stream
        flat = t.view(-1)
        n = flat.numel()
        per = -(-n // self.ws)            # ceil(n / ws)
        chunk = -(-per // 64) * 64         # 64-element multiple: 16-B aligned chunk starts
        bounds = [(min(r * chunk, n), min((r + 1) * chunk, n)) for r in range(self.ws)]
        part = [flat[s:e] for s, e in bounds]
        mine = part[self.me]
        m = mine.numel()
        es = t.element_size()
        scratch = self.cs._scratch(t, (self.ws - 1) * chunk)
        slot = {}
        with stream_ctx(cs):
            if after is not None:
                cs.wait_event(after)
            self._barrier()  # B0
            fork = torch.cuda.Event()
            fork.record(cs)
        joins = []
        peers = [(self.me + d) % self.ws for d in range(1, self.ws)]
        for i, p in enumerate(peers):
            slot[p] = scratch[i * chunk:i * chunk + m]
            if not m:
                continue
            st = self.copy_streams[i]
            with torch.cuda.stream(st):
                st.wait_event(fork)
                mod.copy_from_peer(slot[p], self._peer_addr(t, p) + bounds[self.me][0] * es)
                ev = torch.cuda.Event()
                ev.record(st)
                joins.append(ev)
        with stream_ctx(cs):
            for ev in joins:
                cs.wait_event(ev)
            if m:
                reduce_sum_(mine, [mine if r == self.me else slot[r] for r in range(self.ws)])
            self._barrier()  # B1
            fork = torch.cuda.Event()
            fork.record(cs)
        joins = []
        for i, p in enumerate(peers):
            if not part[p].numel():
                continue
            st = self.copy_streams[i]
            with torch.cuda.stream(st):
                st.wait_event(fork)
                mod.copy_from_peer(part[p], self._peer_addr(t, p) + bounds[p][0] * es)
                ev = torch.cuda.Event()
                ev.record(st)
                joins.append(ev)
        with stream_ctx(cs):
            for ev in joins:
                cs.wait_event(ev)
            self._barrier()  # B2
            if done is not None:
                done.record(cs)

    def _barrier(self) -> None:
        """Stream-ordered on RCCL (one-element all-reduce on the comm stream);
        gloo rehearsal: drain the comm stream, then a host barrier."""
        if self.ws == 1:
            return
        if self.gloo:
            self.cs.stream.synchronize()
            dist.barrier(group=self.group)
        else:
            dist.all_reduce(self.flag, group=self.group)

    def close(self) -> None:
        mod = _mod()
        torch.cuda.synchronize(self.device)
        for _, _, peers in self.bufs:
            for addr in peers.values():
                mod.ipc_close(addr, self.dev_index)
        self.bufs = []
        if self.ws > 1:
            dist.barrier(group=self.group)
