"""GEMM entry points: ``matmul`` / ``bmm`` / ``bench_matmul``.

GPU tensors run on the hand-written gfx950 MFMA kernels of ``ops/csrc``,
chosen per problem by the C++ planner (gemm_dispatch.cpp): bf16/fp16 on
``gemm_w4.hip`` (W4, and its persistent streaming form W4S on a device the
GEMM has to itself), the ``gemm_tile.hip`` family (T128 / T256x128 /
T128x2 / T192 / T192x128, split-K) for grids that under-fill the 256 CUs or
that only 192-row tiles cut into whole waves, SCHED 3 of
``gemm_mfma256.hip`` for edge tiles the others do not take; exact fp32 on
``gemm_f32_w4.hip`` (f32_w4l, the lean K-loop, on whole waves of 256x256
tiles alone on the device), ``gemm_f32_tile.hip`` (f32_t128x2 on other grids of
>= 2 tiles per CU, f32_t128 unsplit on the lean loop or split-K below that, f32_t64 = 64x128 tiles where they fill the chip unsplit, f32_t64x2 = those two per CU, split), ``gemm_f32_256.hip`` and ``gemm_f32_w4.hip`` (split-K)
as the planner prices them; fp8 e4m3 on ``gemm_fp8.hip`` and
the fp8 tile family; ``gemm_generic.hip`` for anything else. Large problems
whose K / N / alignment miss the LDS-DMA granule are zero-padded onto the
fast kernels. CPU tensors use ``torch.matmul`` — the reference's own
compute call (matmul_benchmark.py:46) — which is the BASELINE config #1 CPU
path ("4k fp32 matmul, single process on CPU").

``matmul(..., signal=(SignalSet, rows, epoch))`` runs W4 with per-piece
completion signals: the overlap schedules (parallel/overlap.py) start each
row piece's collective while the rest of the same launch still computes.

Every call writes into a caller-provided (or freshly allocated) ``out``
and is enqueued on the current HIP stream, so it composes with
``torch.cuda.stream(...)`` and events exactly like an ATen op.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

import torch

from . import _native

# The shipping kernels: the public ``kernel=`` surface (api.h ``Kernel``).
KERNELS = {"auto": 0, "generic": 2, "f32_256s": 7, "mfma256d": 9, "fp8_w4": 16, "w4": 21,
           "t128": 26, "t128x2": 27, "t256x128": 28, "f32_w4": 29, "w4s": 36, "fp8_w4s": 37,
           "fp8_t128": 41, "fp8_t256x128": 42, "f32_t128": 51, "f32_t128x2": 53,
           "t192": 60, "t192x128": 61, "fp8_t192": 62, "fp8_t192x128": 63, "f32_t64": 64,
           "f32_t64x2": 65, "f32_w4l": 66}
# A/B and timing-only diagnostic kernels (api.h ``ExperimentKernel``): accepted
# only by a library built with ``PDMB_EXPERIMENTS=1``; ``diag_*`` ones skip waits
# or data movement on purpose and compute WRONG results.
EXPERIMENT_KERNELS = {"mfma256": 1, "mfma256b": 3, "mfma256c": 4, "mfma256c_stamp": 5,
                      "f32_256": 6, "x_clusterprio": 10, "x_staticprio": 11, "x_tall": 13,
                      "fp8": 15, "diag_fp8_w4_nowait": 17, "diag_fp8_w4_nosync": 18,
                      "diag_fp8_w4_mfma_only": 19, "diag_f32_nodma": 20, "x_w4_tall": 22,
                      "x_w4_wide": 23, "x_fp8_w4_tall": 24, "x_fp8_w4_wide": 25,
                      "x_w4_il32": 30, "x_fp8_w4_scaled": 31, "diag_w4_trace": 32,
                      "diag_fp8_w4_trace": 33, "x_w4_pers": 34, "diag_w4_pers_trace": 35,
                      "diag_w4s_trace": 38, "x_w4s_rot": 39, "diag_w4s_rot_trace": 40,
                      "x_fp8_w4_tstore": 43, "x_fp8_w4s_tstore": 44, "x_w4s_tstore": 45,
                      "x_f32_256s_direct": 46, "x_fp8_w4_unfused": 47,
                      "x_t128_unfused": 48, "x_fp8_t128_unfused": 49,
                      "x_w4_unfused": 50, "x_f32_t128_b32": 52, "x_f32_w4_b32": 54,
                      "x_f32_256p": 55, "diag_w4s_nofrag": 56, "diag_w4s_nodma": 57,
                      "diag_w4s_noepi": 58, "diag_w4s_mfma_only": 59, "x_w4s_tall": 70,
                      "x_w4s_wide": 71, "x_w4s_snake": 72, "x_w4s_mcol": 73,
                      "x_fp8_w4s_k4": 74, "x_fp8_w4s_k4_tstore": 75, "x_w4s_st9": 76,
                      "x_w4_st9": 77, "x_fp8_w4s_st9": 78, "x_fp8_w4_st9": 79, "x_f32_w4_nb": 80, "x_f32_w4_nbp": 81,
                      "diag_f32_w4_nodma": 82, "diag_f32_w4_nofrag": 83, "diag_f32_w4_mfma_bar": 84,
                      "diag_f32_w4_mfma_only": 85, "x_f32_w4_spread": 86, "x_f32_w4_spread_dma": 87,
                      "x_f32_w4_spread_rd": 88, "x_f32_w4_lean": 89, "x_f32_w4_lean2": 90, "x_f32_w4s": 91,
                      "x_f32_t128_lean": 92, "x_f32_t128x2_lean": 93, "x_f32_t64_lean": 94,
                      "x_f32_t64x2_lean": 95, "diag_f32_w4s_dbg": 96,
                      "x_w4s_lean": 97, "x_fp8_w4s_thin": 98, "x_w4s_thin": 99}
KERNEL_NAMES = {0: "auto", 2: "pdmb_generic_nn", 7: "pdmb_f32_256s_nn", 9: "pdmb_mfma256d_nn",
                16: "pdmb_fp8_w4_nt", 21: "pdmb_w4_nn", 26: "pdmb_t128_nn",
                27: "pdmb_t128x2_nn", 28: "pdmb_t256x128_nn", 29: "pdmb_f32_w4_nn", 36: "pdmb_w4s",
                37: "pdmb_fp8_w4s", 41: "pdmb_fp8_t128_nt", 42: "pdmb_fp8_t256x128_nt",
                51: "pdmb_f32_t128_nn", 53: "pdmb_f32_t128x2_nn", 60: "pdmb_t192_nn",
                61: "pdmb_t192x128_nn", 62: "pdmb_fp8_t192_nt", 63: "pdmb_fp8_t192x128_nt",
                64: "pdmb_f32_t64_nn", 65: "pdmb_f32_t64x2_nn", 66: "pdmb_f32_w4l_nn",
                1: "pdmb_mfma256_nn",
                3: "pdmb_mfma256b_nn", 4: "pdmb_mfma256c_nn", 5: "pdmb_mfma256c_stamp",
                6: "pdmb_f32_256_nn", 15: "pdmb_fp8_256_nt", -1: "unsupported"}
SUPPORTED_DTYPES = (torch.float32, torch.float16, torch.bfloat16)
FP8 = torch.float8_e4m3fn  # OCP e4m3 (gfx950), bf16 output, column-major B


_budget = threading.local()


@contextlib.contextmanager
def cu_budget(cus: int):
    """GEMMs issued in this block (this thread) run on a stream that may use
    only ``cus`` CUs (a CU-masked stream, parallel/overlap.py): the W4 / T128
    planner sizes their grids for that many CUs instead of the whole device."""
    prev = getattr(_budget, "cus", 0)
    _budget.cus = int(cus)
    try:
        yield
    finally:
        _budget.cus = prev


@contextlib.contextmanager
def shared_device():
    """GEMMs issued in this block (this thread) share the device with
    concurrent kernels (the RCCL collectives of an overlap schedule): the
    planner then keeps to kernels whose tiles the hardware dispatches as CUs
    free up, never a persistent one (W4S) that assumes every CU is its own."""
    prev = getattr(_budget, "shared", False)
    _budget.shared = True
    try:
        yield
    finally:
        _budget.shared = prev


def _cus() -> int:
    """CU budget for the C++ planner: > 0 a masked stream's CUs, 0 the whole
    device to itself, -1 the whole device shared (shared_device)."""
    cus = getattr(_budget, "cus", 0)
    if cus == 0 and getattr(_budget, "shared", False):
        return -1
    return cus


def experiments_built() -> bool:
    """True iff the loaded library carries the experiment kernels."""
    return bool(getattr(_native.load(), "EXPERIMENTS", False))


def _kid(kernel) -> int:
    if isinstance(kernel, int):
        if kernel in KERNELS.values() or (kernel in EXPERIMENT_KERNELS.values()
                                          and experiments_built()):
            return kernel
        raise ValueError(f"kernel id {kernel} is not a shipping kernel of this build")
    if kernel in KERNELS:
        return KERNELS[kernel]
    if kernel in EXPERIMENT_KERNELS:
        if not experiments_built():
            raise ValueError(f"kernel {kernel!r} is an experiment/diagnostic kernel, not built by "
                             "default (rebuild with PDMB_EXPERIMENTS=1 to A/B it)")
        return EXPERIMENT_KERNELS[kernel]
    raise ValueError(f"unknown kernel {kernel!r}; choose from {sorted(KERNELS)}")


def _out_shape(A: torch.Tensor, B: torch.Tensor):
    batch = []
    if A.dim() == 3 or B.dim() == 3:
        batch = [A.shape[0] if A.dim() == 3 else B.shape[0]]
    return (*batch, A.shape[-2], B.shape[-1])


def _prep(t: torch.Tensor) -> torch.Tensor:
    # Kernels need a unit innermost stride and a row stride of at least the row
    # length (no expanded / overlapping rows); leading dims may be strided.
    if t.dim() >= 1 and t.shape[-1] > 1 and t.stride(-1) != 1:
        return t.contiguous()
    if t.dim() >= 2 and t.shape[-2] > 1 and t.stride(-2) < t.shape[-1]:
        return t.contiguous()
    return t


def _prep_colmajor(t: torch.Tensor) -> torch.Tensor:
    # fp8 B operand: unit stride along K (column-major [K,N], i.e. a row-major Bt [N,K]).
    if (t.shape[-2] > 1 and t.stride(-2) != 1) or (t.shape[-1] > 1 and t.stride(-1) < t.shape[-2]):
        return t.transpose(-1, -2).contiguous().transpose(-1, -2)
    return t


def _prep_pair(A: torch.Tensor, B: torch.Tensor):
    if A.dtype == FP8:
        return _prep(A), _prep_colmajor(B)
    return _prep(A), _prep(B)


def out_dtype(dtype: torch.dtype) -> torch.dtype:
    """Output dtype of a native GEMM on ``dtype`` operands (fp8 → bf16)."""
    return torch.bfloat16 if dtype == FP8 else dtype


def fp8_quantize(x: torch.Tensor, colmajor: bool = False):
    """Per-tensor scaled OCP e4m3 copy of ``x``: returns ``(x8, scale)`` with
    ``x ≈ scale * x8.float()`` (amax mapped to 448, e4m3's largest finite).
    ``colmajor=True`` lays the copy out column-major (the fp8 B operand)."""
    amax = x.detach().abs().amax().float().clamp(min=1e-12)
    scale = float(amax) / 448.0
    src = x.transpose(-1, -2) if colmajor else x
    x8 = (src.float() / scale).to(FP8).contiguous()
    return (x8.transpose(-1, -2) if colmajor else x8), scale


class SignalSet:
    """Completion signals of one GEMM output (api.h ``Signal``): ``slots``
    device tile counters plus host-mapped flags. Launch ``e`` (``next_epoch``)
    of a signalled GEMM writes ``e`` into slot s's flag once every tile of
    row piece s is stored (write-through, drained); ``wait`` blocks this host
    thread (GIL released) until then."""

    def __init__(self, device: torch.device, slots: int):
        self._C = _native.load()
        self.device = device
        self.slots = int(slots)
        self.handle = int(self._C.signal_create(device.index, self.slots))
        self.epoch = 0

    def next_epoch(self) -> int:
        self.epoch += 1
        return self.epoch

    def flag(self, slot: int) -> int:
        return int(self._C.signal_flag(self.handle, slot))

    def wait(self, slot: int, epoch: int, timeout_s: float = 30.0) -> None:
        if not self._C.signal_wait(self.handle, int(slot), int(epoch), float(timeout_s)):
            raise TimeoutError(f"GEMM completion signal: slot {slot} did not reach epoch {epoch} "
                               f"within {timeout_s:.0f} s (flag {self.flag(slot)})")

    def set(self, slot: int, value: int) -> None:
        """Host store of slot's flag (opens a ``gate`` waiting for ``value``)."""
        self._C.signal_set(self.handle, int(slot), int(value))

    def gate(self, slot: int, value: int, timeout_s: float = 20.0) -> None:
        """Enqueue on the current stream a one-wave kernel that holds the stream
        until slot's flag reaches ``value`` (``set``) or ``timeout_s`` pass."""
        self._C.gate(self.handle, int(slot), int(value), float(timeout_s))

    def close(self) -> None:
        if self.handle:
            torch.cuda.synchronize(self.device)
            self._C.signal_destroy(self.handle)
            self.handle = 0

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def signal_granule(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
                   kernel="auto") -> int:
    """256-row tile rows of one completion unit of a signalled ``matmul`` (one
    256-workgroup round of W4's tile order); 0 if the problem cannot run
    signalled (not W4, fp8, CPU)."""
    if A.device.type != "cuda" or A.dtype not in (torch.bfloat16, torch.float16):
        return 0
    C = _native.load()
    A, B = _prep_pair(A, B)
    return int(C.signal_granule(A, B, out, _kid(kernel), _cus()))


def matmul(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
           kernel="auto", alpha: float = 1.0, splitk: int = 0, signal=None) -> torch.Tensor:
    """``out = A @ B`` for 2-D/3-D row-major operands (3-D = batched).

    ``splitk`` (W4 / T128 only): K slices per output tile, 0 = auto (split only
    grids that under-fill the 256 CUs, ``splitk_for``), 1 = never.

    ``signal=(SignalSet, rows, epoch)``: run W4 with completion signals, one
    slot per ``rows`` 256-row tile rows (per batch element); raises if the
    problem does not run on W4 (``signal_granule`` == 0).

    float8_e4m3fn operands: ``out = alpha * (A @ B)`` in bfloat16 on the
    block-scaled fp8 MFMA (B is used column-major; a row-major B is copied).
    ``alpha`` folds the per-tensor scales (see ``fp8_quantize``)."""
    if A.dim() not in (2, 3) or B.dim() not in (2, 3):
        raise ValueError("matmul: operands must be 2-D or 3-D")
    if A.shape[-1] != B.shape[-2]:
        raise ValueError(f"matmul: shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")
    if A.device.type != "cuda" and A.dtype == FP8:
        res = (torch.matmul(A.float(), B.float()) * alpha).to(torch.bfloat16)
        if out is None:
            return res
        out.copy_(res)
        return out
    if A.device.type != "cuda":
        if A.dim() == 3 or B.dim() == 3:
            res = torch.matmul(A, B)
            if out is None:
                return res
            out.copy_(res)
            return out
        return torch.matmul(A, B, out=out) if out is not None else torch.matmul(A, B)
    if A.dtype not in SUPPORTED_DTYPES and A.dtype != FP8:
        raise TypeError(f"matmul: unsupported dtype {A.dtype}")
    C = _native.load()
    A, B = _prep_pair(A, B)
    if out is None:
        out = torch.empty(_out_shape(A, B), dtype=out_dtype(A.dtype), device=A.device)
    # auto: odd K/N/alignment padded onto the fast path (C++; not for fp8)
    if signal is not None:
        sig, rows, epoch = signal
        C.matmul(A, B, out, _kid(kernel), float(alpha), int(splitk), _cus(), sig.handle, int(rows),
                 int(epoch))
    else:
        C.matmul(A, B, out, _kid(kernel), float(alpha), int(splitk), _cus())
    return out


PAD_MIN_FLOPS = 2.0 ** 31  # gemm_dispatch.cpp kPadMinFlops


def padded_kernel_for(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None
                      ) -> Optional[str]:
    """Fast kernel an ``auto`` call runs through zero-padded copies, or None
    (under the caller's CU budget / shared-device context, like ``matmul``)."""
    if A.device.type != "cuda" or A.dtype not in SUPPORTED_DTYPES:
        return None
    C = _native.load()
    A, B = _prep_pair(A, B)
    k = int(C.resolve_padded(A, B, out, _cus()))
    return _name(C, k) if k >= 0 else None


def bmm(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
        kernel="auto") -> torch.Tensor:
    """Batched ``out[b] = A[b] @ B[b]`` (the reference's ``torch.bmm``)."""
    if A.dim() != 3 or B.dim() != 3:
        raise ValueError("bmm: operands must be 3-D")
    if A.device.type != "cuda" and A.dtype != FP8:
        return torch.bmm(A, B, out=out) if out is not None else torch.bmm(A, B)
    return matmul(A, B, out=out, kernel=kernel)


def kernel_for(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
               kernel="auto") -> str:
    """Name of the native kernel that ``matmul`` would launch for these operands."""
    if A.device.type != "cuda":
        return "torch.matmul(cpu)"
    C = _native.load()
    A, B = _prep_pair(A, B)
    return _name(C, int(C.resolve(A, B, out, _kid(kernel), _cus())))


def _name(C, k: int) -> str:
    """Kernel name of id ``k`` (the library's own table for ids not mirrored here)."""
    return KERNEL_NAMES.get(k) or str(C.kernel_name(k))


def splitk_for(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
               kernel="auto", splitk: int = 0) -> int:
    """K slices the W4 / T128 kernel uses for these operands (1: unsplit, 0: neither)."""
    if A.device.type != "cuda":
        return 0
    C = _native.load()
    A, B = _prep_pair(A, B)
    return int(C.splitk_for(A, B, out, _kid(kernel), int(splitk), _cus()))


def tail_split_for(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
                   kernel="auto") -> tuple:
    """(M1, S, T1, R): auto runs rows [0, M1) as one W4 launch and the remaining
    tile rows as a second, S-way split-K launch that fills the chip
    (gemm_dispatch.cpp tail_plan), or — the tile-range form, M1 = 0 — the
    first T1 tiles of its tile order (whole waves) as one launch and the rest
    S-way split, or (R > 1, refined tail) the rest cut into R smaller tiles of
    the tile family, unsplit; (0, 1, 0, 1) when the problem runs as one launch."""
    if A.device.type != "cuda":
        return (0, 1, 0, 1)
    C = _native.load()
    A, B = _prep_pair(A, B)
    m1, s, t1, r = C.tail_split_for(A, B, out, _kid(kernel), _cus())
    return (int(m1), int(s), int(t1), int(r))


def bench_matmul(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, iters: int,
                 warmup: int, graph: bool = False, kernel="auto", splitk: int = 0) -> float:
    """Native timing loop (hipEvents around ``iters`` launches). Returns TOTAL ms."""
    if A.device.type != "cuda":
        import time

        for _ in range(warmup):
            matmul(A, B, out=out)
        t0 = time.perf_counter()
        for _ in range(iters):
            matmul(A, B, out=out)
        return (time.perf_counter() - t0) * 1e3
    C = _native.load()
    A, B = _prep_pair(A, B)
    return float(C.bench(A, B, out, int(iters), int(warmup), bool(graph), _kid(kernel),
                         int(splitk)))


def comm_proxy(dst: torch.Tensor, src: torch.Tensor, blocks: int = 32) -> None:
    """Copy ``src`` into ``dst`` on the current stream with exactly ``blocks``
    256-thread workgroups: the CU footprint of an RCCL collective's channels,
    for single-GPU overlap experiments (scripts/cu_mask_overlap.py)."""
    _native.load().comm_proxy(dst, src, int(blocks))


TRACE_KERNELS = {"w4": "diag_w4_trace", "fp8_w4": "diag_fp8_w4_trace", "x_w4_pers": "diag_w4_pers_trace",
                 "w4s": "diag_w4s_trace", "x_w4s_rot": "diag_w4s_rot_trace"}


def tile_trace(A: torch.Tensor, B: torch.Tensor, kernel: str = "w4") -> torch.Tensor:
    """Run one launch of ``kernel``'s tile-timeline build (experiment builds
    only) and return its trace: int64 [workgroups, 8] = start, first K-tile
    in registers, K-loop done, C drained (s_memrealtime, 100 MHz), HW_ID,
    XCC_ID, tm << 32 | tn, 0 (common.h tile_trace_write). Row = blockIdx.x."""
    C = _native.load()
    kid = _kid(TRACE_KERNELS.get(kernel, kernel))
    A, B = _prep_pair(A, B)
    out = torch.empty(_out_shape(A, B), dtype=out_dtype(A.dtype), device=A.device)
    M, N = out.shape[-2], out.shape[-1]
    batch = out.numel() // (M * N)
    blocks = -(-M // 256) * -(-N // 256) * batch
    buf = torch.zeros(blocks, 8, dtype=torch.int64, device=A.device)
    C.set_debug_buffer(buf)
    try:
        C.matmul(A, B, out, kid, 1.0, 0, _cus())
        torch.cuda.synchronize(A.device)
    finally:
        C.set_debug_buffer(None)
    return buf.cpu()
