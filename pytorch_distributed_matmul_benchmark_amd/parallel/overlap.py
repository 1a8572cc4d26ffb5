"""Overlap schedules shared by ``bench.py`` and ``models/``: whole GEMMs on the
compute stream, their collectives on the comm stream, pipelined across units
through a ring of output buffers — and, within a unit, started piece by piece
as the SAME GEMM launch's tiles finish.

Reference: backup/matmul_overlap_benchmark.py:93-180 (two streams, double
buffer: the all-reduce of buffer i runs while buffer i±1 computes; the
collective is issued with no dependency on its producer — SURVEY Q7) and
matmul_scaling_benchmark.py:106-238 (batch_parallel / matrix_parallel,
serialized). Here (``OverlapPipeline``):

* **No chunked GEMM.** Round 2 cut the GEMM into row-chunk launches so a
  chunk's collective could start early; at the ws = 8 shard the 4-chunk GEMM
  ran 977 TF against 1560 unchunked and the overlap lost to serializing
  (profiles/r2_cu_mask_overlap_v2.jsonl). Every unit is now ONE launch of
  the best kernel for the whole problem.
* **Ring of outputs (cross-unit pipelining).** Unit k writes ring buffer
  k % R; its collective runs on the comm stream while unit k+1 computes, and
  unit k+R waits only for unit k's collective (write-after-read), never for
  the most recent one: only the last unit of a timed region is exposed.
  batch_parallel with >= 2 local batch elements rings over its own C[b];
  with one element, and for matrix_parallel, R = 2 (the reference's C1/C2).
* **Signalled pieces (within a unit).** With ``pieces`` > 1 the unit's GEMM
  is the W4 kernel with completion signals (ops/csrc gemm_w4.hip SIG,
  common.h signal_tile): each tile's C leaves write-through, and the tile
  that completes a row piece writes the launch's epoch into that piece's
  host-mapped flag. The host thread — which has already enqueued the next
  unit's GEMM — waits for piece p's flag and issues piece p's collective at
  once, so communication starts while the same launch still computes, with
  no chunk launches, no CU set aside for a polling kernel and no GPU-side
  wait a shared hardware queue could deadlock.
* ``plan_overlap`` prices serial vs overlapped (P pieces) from a GEMM model
  and an xGMI bus-bandwidth model of the collective and refuses plans that
  lose (``OverlapPlan.overlap`` False: the mode runs serialized).
* ``compute_stream(device, comm_cus)`` — optionally a HIP stream whose
  kernels may not use ``comm_cus`` CUs (hipExtStreamCreateWithCUMask, spread
  evenly over the 8 XCDs), so RCCL's workgroups start on those CUs at once.
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .comm import CommStream, new_event, stream_ctx
from .partition import ceil_div


# ---- the planner -------------------------------------------------------------
# GEMM rate (TFLOPS) of a full grid per dtype on one MI355X, measured
# (docs/HISTORY.md headline table: W4 / W4S 16k bf16 1526, fp16 ~ bf16, exact
# fp32 152, fp8 3300); an under-filled grid runs at the fraction of the
# 256 CUs its 256x256 tiles fill (split-K recovers part: floor 0.6).
GEMM_TFLOPS = {torch.bfloat16: 1500.0, torch.float16: 1500.0, torch.float32: 150.0,
               torch.float8_e4m3fn: 3200.0}
# RCCL bus bandwidth (GB/s) by world size on a fully connected 8 x MI355X
# xGMI node (7 links per GPU, ~153 GB/s each; one link between any pair),
# the busBW convention of rccl-tests: t = bytes x factor / busbw with factor
# (ws-1)/ws for all-gather (bytes = gathered total) and 2(ws-1)/ws for
# all-reduce. Defaults are conservative estimates, NOT measured here (no
# multi-GPU node in this build's reach); override with
# PDMB_BUSBW_GBPS="2:80,4:200,8:320" once measured.
DEFAULT_BUSBW_GBPS = {2: 70.0, 4: 180.0, 8: 300.0}
COLLECTIVE_LAT_US = 30.0   # per collective call: host issue + RCCL launch + handshake
PIECE_HOST_US = 15.0       # per signalled piece: host flag latency + issue
RCCL_CU_SHARE = 0.125      # GEMM slowdown while a collective runs beside it (~32 of 256 CUs)


def busbw_gbps(ws: int) -> float:
    env = os.environ.get("PDMB_BUSBW_GBPS", "")
    table = dict(DEFAULT_BUSBW_GBPS)
    for item in filter(None, (x.strip() for x in env.split(","))):
        k, v = item.split(":")
        table[int(k)] = float(v)
    if ws in table:
        return table[ws]
    ks = sorted(table)
    lo = max([k for k in ks if k <= ws], default=ks[0])
    return table[lo]


def gemm_us(m: int, n: int, k: int, dtype: torch.dtype, batch: int = 1) -> float:
    """Model time of one [m, k] @ [k, n] GEMM (x batch) on one MI355X."""
    tiles = ceil_div(max(m, 1), 256) * ceil_div(max(n, 1), 256) * max(batch, 1)
    waves = ceil_div(tiles, 256)
    fill = max(tiles / (waves * 256.0), 0.6)
    return 2.0 * m * n * k * max(batch, 1) / (GEMM_TFLOPS.get(dtype, 1500.0) * 1e6 * fill)


def collective_us(kind: str, payload_bytes: float, ws: int) -> float:
    """Model time of ONE collective on ``payload_bytes`` per rank (all_reduce:
    the reduced tensor; all_gather: this rank's contribution)."""
    if ws <= 1:
        return 0.0
    bw = busbw_gbps(ws) * 1e3  # bytes per us
    if kind == "all_reduce":
        moved = 2.0 * (ws - 1) / ws * payload_bytes
    elif kind == "all_gather":
        moved = (ws - 1) * payload_bytes  # (ws-1)/ws of the gathered total
    else:
        raise ValueError(kind)
    return moved / bw + COLLECTIVE_LAT_US


@dataclass
class OverlapPlan:
    overlap: bool          # False: serialize (the overlap loses or cannot help)
    pieces: int            # collective pieces per unit (1: behind the whole GEMM)
    rows: int              # 256-row tile rows per piece (signal slot; 0 if pieces == 1)
    gemm_us: float
    comm_us: float
    serial_us: float       # predicted per unit, serialized
    overlap_us: float      # predicted per unit, overlapped with the chosen pieces
    candidates: Dict[int, float] = field(default_factory=dict)
    reason: str = ""
    # "measured": gemm_us / comm_us / piece_us timed on this job's ranks (MAX
    # over ranks, measured_plan); "model": the GEMM and busBW tables above
    source: str = "model"
    piece_us: Dict[int, float] = field(default_factory=dict)  # measured: one piece's collective, per P
    # measured: the unit's GEMM while one piece of the P-piece cut runs beside
    # it on the comm stream (``gemm_shared_us``: P = 1, the whole collective),
    # and the slowdown share that implies (``cu_share_p[P]`` = (G'_P - G) /
    # min(G, piece_P): the fraction of the overlapped GEMM time the
    # collective costs; ``cu_share``: P = 1); model: None and RCCL_CU_SHARE
    gemm_shared_us: Optional[float] = None
    cu_share: float = RCCL_CU_SHARE
    cu_share_p: Dict[int, float] = field(default_factory=dict)
    # measured: [min, max] over reps and ranks of every timed value (the
    # planner itself uses the median of each rank's reps, MAX over ranks)
    spread_us: Dict[str, List[float]] = field(default_factory=dict)
    # measured: wall time spent measuring, MAX over ranks (the
    # setup cost every overlapped mode and sweep size pays on every rank)
    planner_s: float = 0.0

    def as_dict(self) -> dict:
        d = asdict(self)
        d["candidates"] = {str(k): round(v, 1) for k, v in self.candidates.items()}
        d["piece_us"] = {str(k): round(v, 1) for k, v in self.piece_us.items()}
        for k in ("gemm_us", "comm_us", "serial_us", "overlap_us"):
            d[k] = round(d[k], 1)
        if d["gemm_shared_us"] is not None:
            d["gemm_shared_us"] = round(d["gemm_shared_us"], 1)
        d["cu_share"] = round(d["cu_share"], 4)
        d["cu_share_p"] = {str(k): round(v, 4) for k, v in self.cu_share_p.items()}
        d["spread_us"] = {k: [round(x, 1) for x in v] for k, v in self.spread_us.items()}
        d["planner_s"] = round(d["planner_s"], 3)
        return d


def plan_overlap(m: int, n: int, k: int, dtype: torch.dtype, ws: int, kind: str,
                 payload_bytes: float, granule: int = 0, steps: int = 10,
                 requested: int = 0, gemm_time_us: Optional[float] = None,
                 comm_time_us: Optional[float] = None,
                 piece_us: float = COLLECTIVE_LAT_US + PIECE_HOST_US,
                 piece_time_us: Optional[Dict[int, float]] = None,
                 source: str = "model", gemm_shared_us: Optional[float] = None,
                 spread_us: Optional[Dict[str, List[float]]] = None,
                 shared_time_us: Optional[Dict[int, float]] = None) -> OverlapPlan:
    """Choose how a unit (one [m, k] @ [k, n] GEMM whose output's collective
    follows) overlaps: serialize, pipeline whole collectives across units
    (pieces = 1), or start P row pieces as the GEMM's tiles finish (P > 1,
    needs ``granule`` > 0: tile rows of one completion unit; P <= the number
    of such units). Per unit, over a timed region of ``steps`` units:

        serial      = G + C
        overlap(P)  = max(G', C') + min(G', C') / P / steps
        G'          = G + s * min(G, C')
        C'          = C + (P - 1) * piece_us   (per extra collective call)

    (the steady state is the slower of the two streams; what is exposed once
    per timed region is the faster stream's first / last piece). ``s`` is the
    share of the overlapped GEMM time the collective beside it costs:
    measured per piece count (``shared_time_us[P]`` = the GEMM timed while
    one piece of the P-piece cut runs beside it: s_P = (G'_P - G) /
    min(G, piece_P), clamped to [0, 1] — a small piece can disturb the GEMM
    less per microsecond than a whole collective, e.g. when its bytes stay
    in the MALL; ``gemm_shared_us`` alone stands for P = 1 and every P) or the
    RCCL_CU_SHARE guess.

    ``requested`` > 0 is an explicit request: P = ``requested`` (clamped to
    what the granule allows), overlapped even where the model predicts a
    loss; 0 lets the planner choose, and it refuses an overlap that does not
    beat serial by 2 % (round 3: 3 % — with measured inputs that refused the
    1-GPU proxy's compute-bound shard row, predicted 2.99 % and measured 3.4 %
    faster overlapped, profiles/r4i_overlap_proxy_measured_plan.jsonl). ``gemm_time_us`` / ``comm_time_us`` replace the
    models (measured values: ``measured_plan``, or the 1-GPU proxy sweep);
    ``piece_time_us[P]`` (measured time of ONE piece's collective when a unit
    is cut into P pieces) replaces C' with P x piece_time_us[P]."""
    G = gemm_time_us if gemm_time_us is not None else gemm_us(m, n, k, dtype)
    C = comm_time_us if comm_time_us is not None else collective_us(kind, payload_bytes, ws)
    serial = G + C
    tm = ceil_div(max(m, 1), 256)
    units = tm // granule if granule > 0 else 1
    choices = piece_choices(m, granule, requested)
    measured = dict(piece_time_us or {})
    shared = dict(shared_time_us or {})
    if gemm_shared_us is not None:
        shared.setdefault(1, gemm_shared_us)
    elif 1 in shared:
        gemm_shared_us = shared[1]

    def share_of(Gs: float, piece: float) -> float:
        return min(max((Gs - G) / min(G, piece), 0.0), 1.0) if min(G, piece) > 0 else 0.0

    shares = {P: share_of(v, measured.get(P, C) if P > 1 else C) for P, v in shared.items()}
    share = shares.get(1, RCCL_CU_SHARE)

    def cost(P: int) -> float:
        Cp = P * measured[P] if P in measured else C + (P - 1) * piece_us
        Gp = G + shares.get(P, share) * min(G, Cp)
        return max(Gp, Cp) + min(Gp, Cp) / P / max(steps, 1)

    cands = {P: cost(P) for P in choices}
    best = min(cands, key=lambda P: (cands[P], P))
    ov = cands[best]
    kw = dict(candidates=cands, source=source, piece_us=measured, gemm_shared_us=gemm_shared_us,
              cu_share=share, cu_share_p=shares, spread_us=dict(spread_us or {}))
    if C <= 0.0:
        return OverlapPlan(False, 1, 0, G, C, serial, serial, reason="no collective (ws = 1)", **kw)
    if ov >= serial * 0.98 and requested <= 0:
        return OverlapPlan(False, 1, 0, G, C, serial, ov,
                           reason=f"overlap predicted {ov:.0f} us vs serial {serial:.0f} us: serialize",
                           **kw)
    rows = 0
    if best > 1:
        rows = ceil_div(units, best) * granule
    why = "requested" if requested > 0 else "planned"
    return OverlapPlan(True, best, rows, G, C, serial, ov,
                       reason=f"{why}: {best} piece(s), {ov:.0f} us vs serial {serial:.0f} us", **kw)


def piece_choices(m: int, granule: int, requested: int = 0) -> List[int]:
    """The piece counts ``plan_overlap`` considers for an m-row unit."""
    tm = ceil_div(max(m, 1), 256)
    units = tm // granule if granule > 0 else 1
    choices = [p for p in (1, 2, 4, 8) if p == 1 or (granule > 0 and p <= units)]
    if requested > 0:
        allowed = [p for p in choices if p <= requested]
        choices = [max(allowed)] if allowed else [1]
    return choices


def piece_span(m: int, granule: int, P: int) -> int:
    """Rows of the first (largest) piece when an m-row unit is cut into P pieces."""
    if P <= 1 or granule <= 0:
        return m
    tm = ceil_div(max(m, 1), 256)
    return min(m, ceil_div(tm // granule, P) * granule * 256)


def _granule(units: Sequence[Tuple], native: bool, owner=None) -> int:
    """The signal granule of unit 0's GEMM as the pipeline would issue it
    (beside collectives: ``gemm.shared_device``, a masked stream's CU budget)."""
    import contextlib

    from ..ops import gemm

    A, B, C = units[0]
    if C.device.type == "cuda" and native and A.dtype in (torch.bfloat16, torch.float16):
        with gemm.shared_device(), (owner.budget() if owner is not None else contextlib.nullcontext()):
            return gemm.signal_granule(A, B, C)
    return 0


def plan_for_units(units: Sequence[Tuple], ws: int, kind: str, payload_bytes: float,
                   native: bool = True, requested: int = 0, steps: int = 10,
                   owner=None) -> OverlapPlan:
    """``plan_overlap`` for a ring of (A, B, out) units from the MODELS: the
    shapes of unit 0 and the signal granule of its GEMM. ``measured_plan`` is
    the one the modes use; this is its fallback."""
    A, B, C = units[0]
    return plan_overlap(C.shape[-2], C.shape[-1], A.shape[-1], A.dtype, ws, kind, payload_bytes,
                        granule=_granule(units, native, owner), steps=steps, requested=requested)


def measured_plan(units: Sequence[Tuple], ctx, kind: str, payload_bytes: float, mm: Callable,
                  piece_collective: Callable[[int, int], None], *, native: bool = True,
                  requested: int = 0, steps: int = 10, compute=None, owner=None,
                  comm: Optional[CommStream] = None, reps: int = 5,
                  piece_prepare: Optional[Callable[[int, int], None]] = None) -> OverlapPlan:
    """``plan_overlap`` from times measured on this job's own ranks — the
    reference judges its serialized and overlapped modes by measured time
    (backup/matmul_overlap_benchmark.py:155-164, matmul_scaling_benchmark.py:
    204-224), so the plan is priced the same way instead of from the busBW
    guesses above:

      * G: unit 0's GEMM, ``reps`` launches on the compute stream in the
        context the pipeline issues it in (``compute_ctx``: shared device,
        a masked stream's CU budget), timed with events;
      * C(P) for every piece count P the planner may choose: one collective
        of the first piece's rows, ``piece_collective(start, stop)`` (the
        mode's own collective — RCCL / direct / ipc — on ring slot 0, issued
        on the comm stream), ``reps`` times after a barrier, each host-timed
        until the comm stream drains (so a piece's host issue cost counts);
      * G'(P): the same GEMM, ``reps`` times, each while one piece of the
        P-piece cut (P = 1: the whole collective) runs beside it on the comm
        stream (the GEMM issued first, the piece right behind it) — the
        GEMM's measured slowdown next to the collective, which replaces the
        RCCL_CU_SHARE guess;
      * each value is the median of this rank's reps, then the MAX over
        ranks, so all ranks hold the same plan and one slow rep on one rank
        does not set it; ``spread_us`` records [min, max] over reps and ranks.

    Every phase is agreed across ranks before the next one starts (``all_ok``
    after the GEMM timing and after each P's local preparation —
    ``piece_prepare(start, stop)``: buffer allocation and the like, no
    collective — before that P's first collective): a rank whose
    GEMM or preparation fails never leaves its peers inside a collective it
    skips; on any failure every rank returns the model plan
    (``plan_for_units``), ``source == "model"``. (A collective that itself
    raises on one rank only cannot be agreed on; the phases before it are
    what can fail alone.) Collective: every rank must call it."""
    import statistics
    import time

    from .dist import all_ok, barrier, reduce_scalar

    t_start = time.perf_counter()
    A, B, C = units[0]
    m, ws, dev = C.shape[-2], ctx.world_size, C.device
    granule = _granule(units, native, owner)
    model = plan_overlap(m, C.shape[-1], A.shape[-1], A.dtype, ws, kind, payload_bytes,
                         granule=granule, steps=steps, requested=requested)
    if ws <= 1:
        return model
    choices = piece_choices(m, granule, requested)
    if 1 not in choices:
        choices = [1] + choices
    cuda = dev.type == "cuda"
    cs = comm or CommStream(dev)
    reps = max(int(reps), 1)
    samples: Dict[str, List[float]] = {}

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    def gemm_reps(beside: Optional[int]) -> List[float]:
        """``reps`` GEMM times (us) on the compute stream, issued back to back
        (the pipeline's steady state; each timed by its own event pair, so a
        host gap between launches is not counted); ``beside``: a collective
        of rows [0, beside) issued right behind each GEMM, which it overlaps."""
        out = []
        if cuda:
            cur = compute if compute is not None else torch.cuda.current_stream(dev)
            evs = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with compute_ctx(compute, owner):
                    e0.record(cur)
                    mm(A, B, C)
                    e1.record(cur)
                evs.append((e0, e1))
                if beside is not None:
                    piece_collective(0, beside)
            cs.synchronize()
            sync()
            return [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
        for _ in range(reps):
            t0 = time.perf_counter()
            mm(A, B, C)
            out.append((time.perf_counter() - t0) * 1e6)
            if beside is not None:
                piece_collective(0, beside)
        return out

    def phase(name: str, fn) -> bool:
        """Run one measuring phase on this rank, then agree (collective)."""
        err = None
        try:
            samples[name] = fn()
        except Exception as e:  # a failed measurement falls back to the model, on every rank alike
            err = f"{type(e).__name__}: {e}"
        if not all_ok(ctx, err is None):
            model.reason += f" (measuring failed in {name}: {err or 'on another rank'})"
            return False
        return True

    def warm_gemm():
        sync()
        with compute_ctx(compute, owner):
            mm(A, B, C)  # first launch outside the timing (kernel selection, workspace)
        sync()
        return gemm_reps(None)

    if not phase("gemm", warm_gemm):
        return model

    def coll_reps(span: int) -> List[float]:
        piece_collective(0, span)  # untimed first call (buffers, communicator paths)
        cs.synchronize()
        sync()
        barrier(ctx)
        out = []
        for _ in range(reps):
            t0 = time.perf_counter()
            piece_collective(0, span)
            cs.synchronize()
            sync()
            out.append((time.perf_counter() - t0) * 1e6)
        return out

    for P in choices:
        span = piece_span(m, granule, P)
        if piece_prepare is not None and not phase(f"prepare{P}", lambda: [piece_prepare(0, span)]):
            return model
        if not phase(f"piece{P}", lambda: coll_reps(span)):
            return model
    for P in choices:
        if not phase(f"gemm_shared{P}", lambda: gemm_reps(piece_span(m, granule, P))):
            return model

    def agreed(name: str) -> float:
        return reduce_scalar(ctx, statistics.median(samples[name]), "max")

    spread = {k: [reduce_scalar(ctx, min(v), "min"), reduce_scalar(ctx, max(v), "max")]
              for k, v in sorted(samples.items()) if not k.startswith("prepare")}
    G = agreed("gemm")
    piece = {P: agreed(f"piece{P}") for P in sorted(choices)}
    Gs = {P: agreed(f"gemm_shared{P}") for P in sorted(choices)}
    out = plan_overlap(m, C.shape[-1], A.shape[-1], A.dtype, ws, kind, payload_bytes,
                       granule=granule, steps=steps, requested=requested, gemm_time_us=G,
                       comm_time_us=piece[1], piece_time_us=piece, source="measured",
                       shared_time_us=Gs, spread_us=spread)
    out.planner_s = reduce_scalar(ctx, time.perf_counter() - t_start, "max")  # agreed: MAX over ranks
    return out


def piece_rows(m: int, rows: int) -> List[Tuple[int, int]]:
    """Row ranges [start, stop) of the pieces: ``rows`` 256-row tile rows each."""
    if rows <= 0:
        return [(0, m)]
    step = rows * 256
    return [(s, min(m, s + step)) for s in range(0, m, step)]


def _xcd_spread(ncu: int, k: int, nxcd: int = 8) -> List[int]:
    """k CU indices spread evenly over the XCDs (HIP CU-mask bit i lands on
    XCD i % nxcd on multi-XCD parts): the first k indices do exactly that.
    Checked on the hardware (runtime/cu_mask_probe.hip,
    profiles/r3zo_cu_mask_placement_probe.jsonl): with bits 0..k-1 off every
    XCD runs on 32 - k/8 CUs, and workgroups still go round-robin, 1/8 to each
    XCD; clearing k bits of one residue class instead starves that one XCD.
    Round 4 re-checked the map bit by bit at W4S occupancy (one 147,968-byte
    LDS workgroup per CU; profiles/r4i_cu_mask_bit_map.jsonl): clearing bit i
    alone takes a CU from XCD i % 8 for every i in 0..31, 64, 128, 192, 255."""
    return list(range(min(max(k, 0), ncu)))


# CUs a compute stream gives up at a time: 4 per XCD. A per-XCD count is not
# enough — inside an XCD the dispatcher does not place workgroups on the free
# CUs alone: with bits 0..7 or 0..15 off (1 or 2 CUs per XCD) a grid of one
# workgroup per usable CU at one-workgroup-per-CU occupancy still stacks 8 / 12
# workgroups behind others (start skew 41 us vs 21 us unmasked), while bits
# 0..31 off leave 28 CUs per XCD and no workgroup late
# (profiles/r4h_cu_mask_w4s_occupancy_probe.jsonl) — round 3's masked-W4S
# collapse. A single cleared bit already makes 1-4 workgroups of its XCD late
# (profiles/r4i_cu_mask_bit_map.jsonl).
MASK_GRANULE = 32


def round_comm_cus(k: int, ncu: int = 256) -> int:
    """``--comm-cus k`` as the compute stream applies it: rounded up to whole
    MASK_GRANULE steps (0 stays 0), at most ncu - MASK_GRANULE."""
    if k <= 0:
        return 0
    return min(-(-k // MASK_GRANULE) * MASK_GRANULE, max(ncu - MASK_GRANULE, 0))


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
    """(stream, owner): the current stream (comm_cus == 0) or a CU-masked one
    keeping ``round_comm_cus(comm_cus)`` CUs free (``owner.excluded``)."""
    if device.type != "cuda":
        return None, None
    if comm_cus <= 0:
        return torch.cuda.current_stream(device), None
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    ms = MaskedStream(device, round_comm_cus(comm_cus, ncu))
    return ms.stream, ms


class OverlapPipeline:
    """The overlap schedule (module docstring): a ring of ``units`` — (A, B,
    out) triples; unit k computes ``units[k % R]`` — whose outputs go through
    ``collective(r, p, start, stop, after, done)`` piece by piece on the comm
    stream. ``step()`` issues ``per_step`` units; ``finish()`` issues what is
    still pending and joins the compute stream behind every collective (call
    it before reading the outputs or stopping a timer).

    ``collective`` must enqueue the collective of rows [start, stop) of ring
    slot r's output on the comm stream after event ``after`` (None: the rows
    are known complete) and record ``done`` behind it (CommStream's
    all_reduce / all_gather_into accept exactly these).

    ``operands(k)`` (optional) returns the (A, B) of unit number k (counting
    from 0 over the pipeline's life) instead of its ring slot's own: the
    ``--check`` runs give every unit a distinct product, so a collective
    that reads a ring slot before its GEMM has rewritten it (or after the
    next one has) sees another unit's bits and the check fails.
    ``slot_unit[r]`` is the unit number that last wrote ring slot r.

    Test-only fault injection (the checks' negative control):
    ``PDMB_TEST_SKIP_READY_WAIT=<cycles>`` issues every collective without
    its producer dependency (no ready event, no signal wait) and delays each
    GEMM by ``<cycles>`` GPU clocks on the compute stream, so the collective
    reliably reads the slot's previous contents."""

    def __init__(self, mm: Callable, units: Sequence[Tuple], collective: Callable,
                 device: torch.device, plan: OverlapPlan, per_step: int = 1,
                 compute=None, owner=None, comm: Optional[CommStream] = None,
                 timeout_s: float = 30.0, operands: Optional[Callable[[int], Tuple]] = None):
        from ..ops import gemm

        self.mm, self.units, self.collective = mm, list(units), collective
        self.operands = operands
        skip = os.environ.get("PDMB_TEST_SKIP_READY_WAIT", "")
        self._skip_cycles = int(skip) if skip else None
        self.R = len(self.units)
        if self.R < 2:
            raise ValueError("OverlapPipeline needs a ring of >= 2 output buffers")
        self.device, self.plan, self.per_step = device, plan, max(1, int(per_step))
        self.compute, self.owner = compute, owner
        self.cs = comm or CommStream(device)
        self.timeout_s = timeout_s
        m = self.units[0][2].shape[-2]
        self.signalled = device.type == "cuda" and plan.pieces > 1 and plan.rows > 0
        self.pieces = piece_rows(m, plan.rows if self.signalled else 0)
        self.sigs = ([gemm.SignalSet(device, len(self.pieces)) for _ in range(self.R)]
                     if self.signalled else None)
        self.ready = [new_event(device) for _ in range(self.R)]
        self.done = [new_event(device) for _ in range(self.R)]
        self.used = [False] * self.R
        self.slot_unit = [-1] * self.R
        self.k = 0
        self.pending: Optional[Tuple[int, int]] = None  # (ring slot, epoch) awaiting its pieces

    def _gemm(self, r: int, k: int) -> Optional[int]:
        from ..ops import gemm

        A, B, out = self.units[r]
        if self.operands is not None:
            A, B = self.operands(k)
        self.slot_unit[r] = k
        with compute_ctx(self.compute, self.owner):
            cur = self.compute if self.compute is not None else None
            if self.used[r] and cur is not None:
                cur.wait_event(self.done[r])  # WAR: the buffer's last collective is done
            if self._skip_cycles and cur is not None:
                torch.cuda._sleep(self._skip_cycles)  # test-only: see the class docstring
            if self.signalled:
                epoch = self.sigs[r].next_epoch()
                gemm.matmul(A, B, out=out, signal=(self.sigs[r], self.plan.rows, epoch))
            else:
                epoch = None
                self.mm(A, B, out)
            self.ready[r].record(cur)
        return epoch

    def _issue(self, r: int, epoch: Optional[int]) -> None:
        last = len(self.pieces) - 1
        for p, (s, e) in enumerate(self.pieces):
            if self._skip_cycles is not None:
                after = None  # test-only: no producer dependency at all
            elif epoch is not None:
                self.sigs[r].wait(p, epoch, self.timeout_s)  # rows [s, e) are stored
                after = None
            else:
                after = self.ready[r]
            self.collective(r, p, s, e, after, self.done[r] if p == last else None)
        self.used[r] = True

    def step(self) -> None:
        for _ in range(self.per_step):
            r, k = self.k % self.R, self.k
            self.k += 1
            epoch = self._gemm(r, k)
            if self.signalled:
                # the next GEMM is queued before this host thread blocks on the
                # previous unit's pieces, so the compute stream never runs dry
                if self.pending is not None:
                    self._issue(*self.pending)
                self.pending = (r, epoch)
            else:
                self._issue(r, None)

    def finish(self) -> None:
        if self.pending is not None:
            self._issue(*self.pending)
            self.pending = None
        if self.compute is not None:
            for r in range(self.R):
                if self.used[r]:
                    self.compute.wait_event(self.done[r])

    def close(self) -> None:
        for s in self.sigs or []:
            s.close()


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


def gather_fn(impl: str, comm) -> Callable:
    """The ``(out, inp, after, done)`` all-gather of ``--allgather impl`` on
    ``comm``: RCCL's ``all_gather_into_tensor`` / the direct P2P group on a
    CommStream, or the peer-memory pull of an IpcGather (parallel/ipc.py; a
    CommStream there means CPU tensors: the direct group stands in)."""
    from .ipc import IpcGather

    if isinstance(comm, IpcGather):
        return comm.all_gather
    if impl in ("direct", "ipc"):
        return comm.all_gather_direct
    return comm.all_gather_into


def make_gatherer(impl: str, device: torch.device, sources=(), comm: Optional[CommStream] = None):
    """The comm object for ``--allgather impl`` / ``--allreduce impl``: an
    IpcGather over ``comm`` with ``sources`` (ipc_empty buffers the inputs
    live in) registered when ``impl == "ipc"`` on a GPU, else the CommStream
    itself."""
    from .ipc import IpcGather

    cs = comm or CommStream(device)
    if impl == "ipc" and device.type == "cuda":
        ig = IpcGather(cs)
        try:
            for src in sources:
                ig.register(src)  # fails on every rank together (IpcGather.register)
        except Exception:
            ig.close(barrier=False)  # unmap what the earlier buffers mapped
            raise
        return ig
    return cs


def all_gather_now(out: torch.Tensor, inp: torch.Tensor, impl: str = "rccl", comm=None) -> None:
    """Serialized all-gather on the current stream: RCCL's
    ``all_gather_into_tensor``, or (``comm``: a CommStream / IpcGather from
    ``make_gatherer``) the direct P2P group or the peer-memory pull, with the
    current stream joined behind it."""
    import torch.distributed as dist

    if impl == "rccl":
        dist.all_gather_into_tensor(out, inp)
        return
    dev = inp.device
    cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    ready, done = new_event(dev), new_event(dev)
    ready.record(cur)
    gather_fn(impl, comm)(out, inp, after=ready, done=done)
    if cur is not None:
        cur.wait_event(done)


def reduce_fn(impl: str, comm) -> Callable:
    """The ``(t, after, done)`` SUM all-reduce of ``--allreduce impl`` on
    ``comm``: RCCL's on a CommStream, the direct P2P two-shot exchange, or the
    peer-memory form of an IpcGather (a CommStream there — CPU tensors, or a
    mode without registered outputs — runs the direct exchange)."""
    from .ipc import IpcGather

    if isinstance(comm, IpcGather):
        return comm.all_reduce
    if impl in ("direct", "ipc"):
        return comm.all_reduce_direct
    return comm.all_reduce


def all_reduce_now(t: torch.Tensor, impl: str = "rccl", comm=None) -> None:
    """Serialized SUM all-reduce on the current stream: RCCL's ``all_reduce``,
    or (``comm``: a CommStream / IpcGather) the direct two-shot exchange or
    its peer-memory form, with the current stream joined behind it."""
    import torch.distributed as dist

    if impl == "rccl":
        dist.all_reduce(t)
        return
    dev = t.device
    cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    ready, done = new_event(dev), new_event(dev)
    ready.record(cur)
    reduce_fn(impl, comm)(t, after=ready, done=done)
    if cur is not None:
        cur.wait_event(done)


COLLECTIVE_IMPLS = ("rccl", "direct", "ipc")


def auto_candidates(device: torch.device) -> Tuple[str, ...]:
    """What ``auto`` times: RCCL's collective and the direct P2P exchange (both
    RCCL kernels); the peer-memory pull (parallel/ipc.py) joins only with
    ``PDMB_AUTO_IPC=1``. Every pull it has ever made ran between ranks that
    share ONE GPU (gloo rehearsals): no byte has crossed xGMI between two
    physical devices yet, and a hipErrorIllegalAddress inside a peer pull
    would take every rank down rather than drop the candidate. Once a 2- or
    8-GPU run of the overlapped modes has passed its checks with it
    (``check_collective`` below and bench.py's per-mode check), it can be a
    default candidate again."""
    if device.type == "cuda" and os.environ.get("PDMB_AUTO_IPC", "0") == "1":
        return COLLECTIVE_IMPLS
    return ("rccl", "direct")


def ipc_buffers(impl: str, device: torch.device) -> bool:
    """Whether a mode's collective buffers must be IPC-exportable (``ipc_empty``):
    ``--... ipc``, or ``auto`` with the peer-memory pull among its candidates."""
    return device.type == "cuda" and (impl == "ipc" or (impl == "auto" and "ipc" in auto_candidates(device)))


def pick_collective(ctx, kind: str, t: torch.Tensor, sources=(), comm: Optional[CommStream] = None,
                    reps: int = 5, candidates: Optional[Sequence[str]] = None,
                    spread_out: Optional[Dict[str, List[float]]] = None,
                    _test_corrupt: Optional[Callable[[str, torch.Tensor], None]] = None):
    """``--allreduce auto`` / ``--allgather auto``: time one whole collective of
    ``t`` (all_reduce: in place; all_gather: ``t`` is this rank's block) with
    every candidate implementation on this job's own ranks (``auto_candidates``:
    RCCL's, the direct P2P exchange, and with PDMB_AUTO_IPC=1 the peer-memory
    pull with ``sources`` registered). Each candidate is first CHECKED: two
    calls on rank-coded payloads (parallel/verify.py ``check_collective``),
    compared bitwise with the expected gather / sum; a candidate wrong on any
    rank is dropped on every rank and recorded as ``"wrong"``. Then it is
    timed: ``reps`` reps after a barrier, each timed alone, the median of a
    rank's reps and the MAX over ranks (``spread_out``, if given, receives
    [min, max] over reps and ranks per candidate); the fastest is kept. A
    candidate that raises on any rank is dropped on every rank (``None``).
    ``t``'s contents are overwritten. Returns ``(impl, comm_object, {impl: us
    | None | "wrong"})``; the comm object is what ``make_gatherer(impl, ...)``
    would have built (on ``comm``), the losers' are closed. ``_test_corrupt
    (impl, result)`` (tests only: the gate's negative control) damages a
    checked result on the calling rank. Collective: every rank must call it."""
    import statistics
    import time

    from .dist import all_ok, barrier, reduce_scalar
    from .verify import check_collective

    dev = t.device
    cuda = dev.type == "cuda"
    if candidates is None:
        candidates = auto_candidates(dev)
    cands = list(candidates)
    out = (torch.empty((ctx.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
           if kind == "all_gather" else None)

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    def call(impl, g):
        if kind == "all_reduce":
            all_reduce_now(t, impl, g)
        else:
            all_gather_now(out, t, impl, g)

    times, objs, spread = {}, {}, {}

    def drop(impl, g):  # the candidate is out, on every rank
        times[impl] = None
        if g is not None and hasattr(g, "close"):
            g.close(barrier=False)
        barrier(ctx)

    for impl in cands:
        g, err = None, None
        try:  # built everywhere before any rank enters its collective
            g = make_gatherer(impl, dev, sources, comm=comm or CommStream(dev))
        except Exception as e:  # e.g. no peer access
            err = f"{type(e).__name__}: {e}"
        if not all_ok(ctx, err is None):
            drop(impl, g)
            continue
        wrong = None
        try:
            corrupt = ((lambda res, _i=impl: _test_corrupt(_i, res)) if _test_corrupt is not None
                       else None)
            wrong = check_collective(kind, ctx.rank, ctx.world_size, t, out, lambda: call(impl, g),
                                     sync, corrupt=corrupt)
        except Exception as e:
            err = f"{type(e).__name__}: {e}"
        if not all_ok(ctx, err is None):
            drop(impl, g)
            continue
        if not all_ok(ctx, wrong is None):
            if wrong is not None:
                import sys

                print(f"[rank {ctx.rank}] {kind} candidate {impl!r} returned wrong data: {wrong}",
                      file=sys.stderr, flush=True)
            drop(impl, g)
            times[impl] = "wrong"
            continue
        barrier(ctx)
        reps_us = []
        for _ in range(reps):
            t0 = time.perf_counter()
            call(impl, g)
            sync()
            reps_us.append((time.perf_counter() - t0) * 1e6)
        # median of this rank's reps, MAX over ranks; [min, max] over reps and ranks
        times[impl] = reduce_scalar(ctx, statistics.median(reps_us), "max")
        spread[impl] = [reduce_scalar(ctx, min(reps_us), "min"), reduce_scalar(ctx, max(reps_us), "max")]
        objs[impl] = g
    ok = {k: v for k, v in times.items() if isinstance(v, float)}
    if not ok:
        raise RuntimeError(f"no {kind} implementation ran correctly on every rank: {times}")
    best = min(ok, key=ok.get)
    for impl, g in objs.items():
        if impl != best and hasattr(g, "close"):
            g.close()
    if spread_out is not None:
        spread_out.update({k: [round(x, 1) for x in v] for k, v in spread.items()})
    return best, objs[best], {k: (round(v, 1) if isinstance(v, float) else v) for k, v in times.items()}
