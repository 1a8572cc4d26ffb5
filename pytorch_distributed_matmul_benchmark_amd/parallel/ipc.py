"""Collectives over xGMI peer memory (``--allgather ipc``, ``--allreduce ipc``).

Every rank maps its peers' output buffers once (``hipIpcOpenMemHandle``) and
then PULLS what it needs straight out of their memory: on a fully connected
8 x MI355X node each peer sits behind its own xGMI link, so a pull from all
seven peers drives all seven links at once with no forwarding hop (RCCL's
ring all-gather forwards every block ws - 1 times, one link per hop).

SURVEY §7.2 (K5-K7 stretch): "custom xGMI peer-memory all-gather (hipIpc
handles, 7 links in parallel)"; the reference's all-gather call site is
matmul_scaling_benchmark.py:221 (NCCL ``all_gather``).

Two copy engines (``PDMB_IPC_ENGINE``):

  * ``kernel`` (default): ONE launch on the comm stream does every pull
    (ops/csrc reduce.hip ``multi_copy``: blockIdx.y = peer, 32 workgroups
    per peer by default, ``PDMB_IPC_BLOCKS``), and the all-reduce's sum reads
    its chunk straight out of every peer's buffer (``reduce_sum`` over peer
    addresses: pull and sum fused, no landing copy). It uses CUs — about as
    many workgroups as RCCL's channels — but adds no streams: a rank runs its
    compute stream, the comm stream and RCCL's internal stream, inside the
    process's 4 hardware queues (``GPU_MAX_HW_QUEUES``).
  * ``sdma``: ``hipMemcpyDeviceToDeviceNoCU`` copies (the DMA engines, no
    CU; a plain DeviceToDevice copy runs the runtime's blit kernel) spread
    over at most two copy streams (``COPY_STREAMS``), so the rank stays at
    five streams: copies on one stream run one after another, which is the
    price of the bounded stream count.

Ordering (both engines; every barrier is stream-ordered — a one-element
RCCL all-reduce on the comm stream, whose completion on a rank means every
peer's comm stream has passed the same point):

  * ``all_gather(out, inp, after, done)``: wait ``after`` -> B0 (every
    rank's ``inp`` is final before anyone reads it) -> pull every peer's
    block (same offset in ITS buffer) into ``out``, copy the local one ->
    B1 (every peer has finished reading this rank's block, so its next
    producer may overwrite it) -> record ``done``.
  * ``all_reduce(t, after, done)``: B0 -> this rank's chunk = the sum in rank
    order of that chunk of every rank's ``t`` -> B1 (every chunk reduced) ->
    pull every peer's reduced chunk into place -> B2.

Visibility of a peer's data (why the kernel engine's plain loads are used):
every pull is a NEW kernel launch that starts after B0 has completed on
this rank, and B0 completes only after every peer's comm stream passed its
own B0, which is queued behind that peer's producer kernel. A producer's
writes leave its XCD L2s at the end of its kernel: the per-XCD L2s are not
coherent even within one GPU (docs/guides: MI355X_MICROARCH "Workgroup
dispatch ... inter-workgroup visibility"), so the end-of-kernel release
writes dirty lines back to memory for any later kernel on another XCD, the
same write-back a peer's xGMI read relies on; the pulling kernel's own
start-of-kernel acquire leaves no stale line in its L1/L2. So no in-kernel
fence or system-scope load is needed — one hand-off per kernel boundary,
nothing spins on a flag. This is an argument from the single-GPU memory
model, not a measurement across two physical GPUs: the pull stays out of
``auto`` by default (parallel/overlap.py ``auto_candidates``), and whenever it
runs, ``pick_collective`` has first checked it bitwise on two rank-coded
payloads in a row and bench.py checks every mode's delivered data
(parallel/verify.py), so a stale pull is reported, never timed as correct.

``register(src)`` exports ``src`` (an ``ipc_empty`` tensor: its own
hipMalloc allocation) and maps every peer's counterpart (handles exchanged by
a host all-gather of objects); every rank registers corresponding buffers in
the same order. Exported buffers and peer mappings live until the process
exits (the arena below); ``close()`` drains and barriers.

gloo rehearsals (ranks sharing one GPU) exchange handles the same way; a
barrier becomes "drain the comm stream, then a host barrier". CPU tensors
have no peer memory: ``--allgather ipc`` runs the direct P2P exchange there
(parallel/comm.py).
"""
from __future__ import annotations

import atexit
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .comm import CommStream, stream_ctx


def _mod():
    from ..ops import _native

    return _native.load(build_if_missing=False)


# Process-lifetime IPC arena (default; PDMB_IPC_ARENA=0 bypasses it): the
# native pool (ops/csrc bindings.cpp ``ipc_empty``) never frees an exported
# buffer before exit — a released one returns to the pool and is handed out
# again for the next buffer of its size, under the same cached handle — and
# every peer buffer this process maps stays mapped, opened once per handle
# (``_MAPPED``). So one handle always names one live buffer, a peer's mapping
# of it never goes stale, and nothing is unmapped or freed between benchmark
# modes. The pool holds each distinct (size, device) a process ever exported
# at once — a mode's ring and output buffers, re-used by later modes and
# sweep sizes of the same shapes; a sweep over N sizes holds the buffers of
# all N (about 1.2 GB per size at 16k, ws = 8). With the arena bypassed
# (diagnosis / tests), ``close()`` unmaps this gatherer's peer buffers and a
# released buffer is hipFree'd: the pre-arena behaviour.
_MAPPED: Dict[Tuple[int, bytes], int] = {}  # arena: (device, peer handle) -> mapped address


def arena() -> bool:
    return os.environ.get("PDMB_IPC_ARENA", "1") != "0"


def _release_arena() -> None:
    """atexit: drain the devices and unmap every peer buffer while the HIP
    runtime is still whole, instead of leaving open peer mappings to the
    runtime's static destructors. By exit every collective has completed (the
    process group was torn down after a barrier); a peer that still maps this
    process's memory keeps it alive (dma-buf IPC). (A 2-rank run under
    rocprofv3 crashed in __cxa_finalize with or without IPC — rocprofv3's
    shared output database, not this: per-process ``-o x_%pid%`` avoids it;
    profiles/r4t_rocprof_ipc2_exit_segv.log.)"""
    if not _MAPPED:
        return
    try:
        mod = _mod()
        for d in {dev for dev, _ in _MAPPED}:
            torch.cuda.synchronize(d)
        for (dev, _), addr in list(_MAPPED.items()):
            try:
                mod.ipc_close(addr, dev)
            except Exception:
                pass
    except Exception:
        pass
    _MAPPED.clear()


atexit.register(_release_arena)


def ipc_empty(shape, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """A GPU tensor in its own allocation (IPC-exportable), from the
    process-lifetime pool (above); CPU: plain empty."""
    if device.type != "cuda":
        return torch.empty(shape, dtype=dtype, device=device)
    return _mod().ipc_empty(list(shape), dtype, device.index if device.index is not None else 0)


def _open(mod, handle: bytes, dev_index: int) -> int:
    if not arena():
        return mod.ipc_open(handle, dev_index)
    key = (dev_index, handle)
    if key not in _MAPPED:
        _MAPPED[key] = mod.ipc_open(handle, dev_index)
    return _MAPPED[key]


def checking() -> bool:
    """PDMB_IPC_CHECK=1: every pull / in-place sum is bounds-checked on the host
    before its launch (``IpcGather._check``)."""
    return os.environ.get("PDMB_IPC_CHECK") == "1"


ENGINES = ("kernel", "sdma")
COPY_STREAMS = 2  # sdma engine: copy streams per rank (compute + comm + RCCL + 2 = 5)


def engine() -> str:
    e = os.environ.get("PDMB_IPC_ENGINE", "kernel")
    if e not in ENGINES:
        raise ValueError(f"PDMB_IPC_ENGINE={e!r}: one of {ENGINES}")
    return e


_TRACE = os.environ.get("PDMB_IPC_TRACE") == "1"


def _trace(msg: str) -> None:
    """Diagnostics (PDMB_IPC_TRACE=1): one line per IPC operation on stderr."""
    if _TRACE:
        import sys

        print(f"[ipc pid {os.getpid()}] {msg}", file=sys.stderr, flush=True)


def blocks_per_peer() -> int:
    return int(os.environ.get("PDMB_IPC_BLOCKS", "0"))  # 0: the kernel's default (32)


class IpcGather:
    """Peer-memory all-gather / all-reduce on a CommStream (module docstring)."""

    def __init__(self, comm: CommStream, group=None, engine_name: Optional[str] = None):
        self.cs = comm
        self.group = group
        self.device = comm.device
        self.ws = dist.get_world_size(group)
        self.me = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.engine = engine_name or engine()
        if self.engine not in ENGINES:
            raise ValueError(f"IpcGather engine {self.engine!r}: one of {ENGINES}")
        self.blocks = blocks_per_peer()
        # registered buffers: (local base address, bytes, {peer rank: mapped
        # address}, {peer rank: the peer's buffer bytes})
        self.bufs: List[Tuple[int, int, Dict[int, int], Dict[int, int]]] = []
        self.check = checking()
        self.copy_streams = ([torch.cuda.Stream(device=self.device)
                              for _ in range(min(COPY_STREAMS, max(self.ws - 1, 0)))]
                             if self.engine == "sdma" else [])
        self.flag = torch.zeros(1, device=self.device)
        # test-only fault injection (tests/test_ipc_gpu.py negative control):
        # skip the pre-read barrier B0 so a pull can see a peer's previous data
        self._skip_b0 = os.environ.get("PDMB_TEST_IPC_SKIP_B0") == "1"

    def register(self, src: torch.Tensor) -> None:
        """Export ``src`` and map every peer's corresponding buffer (collective)."""
        assert src.is_cuda and src.storage_offset() == 0, "register an ipc_empty tensor"
        mod = _mod()
        nbytes = src.untyped_storage().nbytes()
        try:
            mine = (mod.ipc_handle(src), nbytes)
        except Exception as e:  # still join the exchange below, so no peer is left waiting
            mine, why = None, e
        handles: List[Optional[Tuple[bytes, int]]] = [None] * self.ws
        dist.all_gather_object(handles, mine, group=self.group)
        if any(h is None for h in handles):
            raise RuntimeError(f"IpcGather: a rank could not export its buffer"
                               f"{f' ({why!r})' if mine is None else ''}")
        peers, sizes, err = {}, {}, None
        try:
            for r, (h, nb) in enumerate(handles):
                if r != self.me:
                    peers[r] = _open(mod, h, self.dev_index)
                    sizes[r] = nb
        except Exception as e:
            err = e
        oks: List[Optional[bool]] = [None] * self.ws  # every rank fails together, or none does
        dist.all_gather_object(oks, err is None, group=self.group)
        if not all(oks):
            if not arena():
                for a in peers.values():
                    mod.ipc_close(a, self.dev_index)
            raise RuntimeError(f"IpcGather: mapping a peer's buffer failed on rank(s) "
                               f"{[r for r, ok in enumerate(oks) if not ok]}"
                               f"{f' ({err!r})' if err is not None else ''}")
        self.bufs.append((src.data_ptr(), nbytes, peers, sizes))
        _trace(f"rank {self.me} register {src.data_ptr():#x} +{nbytes} handle "
               f"{handles[self.me][0][:16].hex()} peers "
               f"{{{', '.join(f'{r}: {a:#x}+{sizes[r]}' for r, a in peers.items())}}}")

    @property
    def npeers(self) -> int:
        """Peers whose buffers are mapped (ws - 1 once a buffer is registered)."""
        return len(self.bufs[0][2]) if self.bufs else 0

    def _peer_addr(self, t: torch.Tensor, peer: int) -> int:
        """Address of ``t``'s counterpart in ``peer``'s buffer (``t`` itself for this rank)."""
        p = t.data_ptr()
        if peer == self.me:
            return p
        for base, nbytes, peers, _ in self.bufs:
            if base <= p and p + t.nbytes <= base + nbytes:
                return peers[peer] + (p - base)
        raise ValueError("IpcGather: the input is not inside a registered buffer")

    def _check(self, what: str, dst: torch.Tensor, src: int, nbytes: int) -> None:
        """PDMB_IPC_CHECK=1 (host side, before the launch): ``src`` +
        ``nbytes`` must lie inside one registered peer extent (the peer's own
        buffer size, exchanged at registration) — or inside this rank's own
        registered buffer — and both ranges inside a live allocation /
        mapping of this process (ops ``ipc_range``: a closed mapping or a
        freed buffer is refused); a violation names the peer, the offset and
        the extent."""
        mod = _mod()
        where = None
        for base, nb, peers, sizes in self.bufs:
            if base <= src < base + nb:
                if src + nbytes > base + nb:
                    raise RuntimeError(
                        f"IpcGather[{what}]: read of {nbytes} B from this rank ({self.me}) at offset "
                        f"{src - base} runs past its own buffer (extent {nb} B)")
                where = (self.me, src - base, nb)
                break
            for r, a in peers.items():
                if a <= src < a + sizes[r]:
                    if src + nbytes > a + sizes[r]:
                        raise RuntimeError(
                            f"IpcGather[{what}]: pull of {nbytes} B from peer {r} at offset "
                            f"{src - a} runs past its buffer (extent {sizes[r]} B)")
                    where = (r, src - a, sizes[r])
                    break
            if where:
                break
        if where is None and nbytes:
            raise RuntimeError(f"IpcGather[{what}]: source {src:#x} (+{nbytes} B) is in no registered "
                               f"buffer of this rank or any peer")
        for addr, n, label in ((src, nbytes, f"source (peer {where[0]}, offset {where[1]}, "
                                             f"extent {where[2]})" if where else "source"),
                               (dst.data_ptr(), dst.nbytes, "destination")):
            if not n:
                continue
            try:
                b, sz = mod.ipc_range(addr, self.dev_index)
            except RuntimeError as e:
                raise RuntimeError(f"IpcGather[{what}]: {label} {addr:#x} +{n} B: {e}") from None
            if addr + n > b + sz:
                raise RuntimeError(f"IpcGather[{what}]: {label} {addr:#x} +{n} B runs past its "
                                   f"allocation [{b:#x}, +{sz})")

    def _pull(self, jobs) -> None:
        """Issue ``jobs`` [(dst tensor, src address)] on the comm stream (kernel
        engine: one launch) or over the copy streams forked from / joined back
        to it (sdma engine). Call with the comm stream current."""
        jobs = [(d, a) for d, a in jobs if d.numel()]
        if not jobs:
            return
        mod = _mod()
        cs = self.cs.stream
        _trace(f"rank {self.me} pull " + ", ".join(f"{d.data_ptr():#x}<-{a:#x}+{d.nbytes}" for d, a in jobs))
        if self.check:
            for d, a in jobs:
                self._check("pull", d, a, d.nbytes)
        if self.engine == "kernel":
            mod.peer_copy([d for d, _ in jobs], [a for _, a in jobs], self.blocks)
            return
        fork = torch.cuda.Event()
        fork.record(cs)
        joins = []
        for i, st in enumerate(self.copy_streams):
            mine = jobs[i::len(self.copy_streams)]
            if not mine:
                continue
            with torch.cuda.stream(st):
                st.wait_event(fork)
                for d, a in mine:
                    mod.copy_from_peer(d, a, True)
                ev = torch.cuda.Event()
                ev.record(st)
                joins.append(ev)
        for ev in joins:
            cs.wait_event(ev)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, after=None, done=None) -> None:
        """``out`` [ws * rows, ...] (contiguous) <- every rank's ``inp`` [rows, ...]."""
        assert inp.is_contiguous() and out.is_contiguous()
        rows = inp.shape[0]
        blocks = [out[r * rows:(r + 1) * rows] for r in range(self.ws)]
        cs = self.cs.stream
        with stream_ctx(cs):
            if after is not None:
                cs.wait_event(after)
            if not self._skip_b0:
                self._barrier()  # B0: every rank's block is final
            # this rank's own block goes through the same engine (sdma: a NoCU
            # copy; a torch copy_ would be the runtime's blit kernel)
            jobs = [(blocks[self.me], inp.data_ptr())]
            jobs += [(blocks[p], self._peer_addr(inp, p))
                     for p in ((self.me + d) % self.ws for d in range(1, self.ws))]
            self._pull(jobs)
            self._barrier()  # B1: no peer still reads this rank's block
            if done is not None:
                done.record(cs)

    def all_reduce(self, t: torch.Tensor, after=None, done=None) -> None:
        """SUM all-reduce of ``t`` (a contiguous view into a registered buffer,
        the same offsets on every rank) over peer memory — the two-shot
        exchange of ``CommStream.all_reduce_direct`` with pulls instead of
        P2P sends (module docstring). Chunks are 64-element multiples (16-B
        aligned); every rank sums in rank order, so all ranks hold identical
        bits."""
        from .comm import reduce_sum_

        assert t.is_contiguous()
        cs = self.cs.stream
        if self.ws == 1 or t.numel() == 0:
            with stream_ctx(cs):
                if after is not None:
                    cs.wait_event(after)
                if done is not None:
                    done.record(cs)
            return
        mod = _mod()
        flat = t.view(-1)
        n = flat.numel()
        per = -(-n // self.ws)            # ceil(n / ws)
        chunk = -(-per // 64) * 64         # 64-element multiple: 16-B aligned chunk starts
        bounds = [(min(r * chunk, n), min((r + 1) * chunk, n)) for r in range(self.ws)]
        part = [flat[s:e] for s, e in bounds]
        mine = part[self.me]
        m = mine.numel()
        es = t.element_size()
        peers = [(self.me + d) % self.ws for d in range(1, self.ws)]
        with stream_ctx(cs):
            if after is not None:
                cs.wait_event(after)
            self._barrier()  # B0: every rank's t is final
            if m:
                if self.engine == "kernel":
                    # pull and sum fused: this chunk of every rank's t, read in place
                    addrs = [self._peer_addr(t, r) + bounds[self.me][0] * es for r in range(self.ws)]
                    _trace(f"rank {self.me} reduce {mine.data_ptr():#x}+{mine.nbytes} <- "
                           + ", ".join(f"{a:#x}" for a in addrs))
                    if self.check:
                        for a in addrs:
                            self._check("reduce", mine, a, mine.nbytes)
                    mod.reduce_sum_addrs(mine, addrs, 0)
                else:
                    scratch = self.cs._scratch(t, (self.ws - 1) * chunk)
                    slot = {p: scratch[i * chunk:i * chunk + m] for i, p in enumerate(peers)}
                    self._pull([(slot[p], self._peer_addr(t, p) + bounds[self.me][0] * es)
                                for p in peers])
                    reduce_sum_(mine, [mine if r == self.me else slot[r] for r in range(self.ws)])
            self._barrier()  # B1: every chunk reduced
            self._pull([(part[p], self._peer_addr(t, p) + bounds[p][0] * es) for p in peers])
            self._barrier()  # B2: no peer still reads this rank's chunk
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

    def close(self, barrier: bool = True) -> None:
        """Finish with this gatherer: drain the device, then (``barrier``) wait
        for every rank to have done so, so no rank's next mode starts while a
        peer still pulls from this one's buffers; ``barrier=False`` when not
        every rank holds a gatherer (the caller runs a common barrier). With
        the arena the mappings stay open for the process; bypassed
        (PDMB_IPC_ARENA=0), this gatherer's peer mappings are closed here,
        after the drain and before the barrier (the pre-arena order)."""
        torch.cuda.synchronize(self.device)
        _trace(f"rank {self.me} close {len(self.bufs)} buffer(s)")
        if not arena():
            mod = _mod()
            for _, _, peers, _ in self.bufs:
                for a in peers.values():
                    mod.ipc_close(a, self.dev_index)
        self.bufs = []
        if barrier and self.ws > 1:
            dist.barrier(group=self.group)
