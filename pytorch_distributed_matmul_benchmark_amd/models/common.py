"""Shared pieces of every workload ("mode"): config, result, GEMM dispatch,
seeded operand generation and the correctness check.

A workload here is the reference's ``benchmark_*`` function
(matmul_scaling_benchmark.py:69-238, backup/matmul_distributed_benchmark.py:
35-174, backup/matmul_overlap_benchmark.py:36-278): allocate seeded random
operands, warm up, align ranks, run the timed loop, return times + FLOPs.

GEMMs on GPU run on this package's gfx950 MFMA kernels (``ops.gemm``), not
on torch.matmul/hipBLASLt; ``backend="torch"`` exists only to A/B against
the vendor library. All outputs are preallocated (the reference allocates a
new C — and a new gather list — every iteration).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import torch

from ..ops import gemm as _gemm
from ..parallel.dist import DistContext, barrier
from ..utils.timing import synchronize


@dataclass
class Workload:
    n: int
    dtype: torch.dtype = torch.bfloat16
    iters: int = 50
    warmup: int = 10
    seed: int = 0
    backend: str = "native"     # native (gfx950 MFMA kernels) | torch (vendor BLAS, for A/B only)
    kernel: str = "auto"        # native kernel selection (auto | mfma256 | generic)
    batch: int = 4              # batch_parallel requested global batch (rounded up to a multiple of ws)
    overlap: bool = False       # comm/compute overlap on a second stream
    chunks: int = 0             # overlap: collective pieces per GEMM (signalled; 0 = planner, 1 = whole)
    comm_cus: int = 0           # overlap: CUs kept free of GEMM workgroups for RCCL (CU-masked stream)
    allgather: str = "rccl"     # matrix_parallel all-gather: rccl | direct (P2P to every peer at once)
    allreduce: str = "rccl"     # all-reduce: rccl | direct (two-shot over P2P links, native sum)
    graph: bool = False         # independent: replay the timed loop as one hipGraph
    check: bool = False         # verify the result against a float64 reference
    min_warmup_ms: float = 0.0  # extend the warm-up until this much GPU time has run (DVFS)


@dataclass
class ModeResult:
    mode: str
    n: int
    world_size: int
    avg_ms: float                     # per-iteration time on this rank
    flops_local: float                # FLOPs this rank executes per iteration
    flops_total: float                # FLOPs all ranks execute per iteration
    tflops: float                     # this rank's TFLOPS, mode-specific definition (see each mode)
    compute_ms: Optional[float] = None
    comm_ms: Optional[float] = None
    compute_only_tflops: Optional[float] = None
    relerr: Optional[float] = None
    kernel: str = ""
    extra: Dict[str, object] = field(default_factory=dict)


def gemm_fn(w: Workload, device: torch.device) -> Callable:
    """``mm(A, B, out)`` for this workload's device/backend (2-D or batched 3-D)."""
    if w.dtype == _gemm.FP8 and (device.type != "cuda" or w.backend == "torch"):
        if device.type != "cuda":
            return lambda A, B, out: _gemm.matmul(A, B, out=out)  # float64-exact dequant path
        one = torch.ones((), device=device)

        def mm(A, B, out):  # hipBLASLt fp8 (A/B only)
            if A.dim() == 3:
                for b in range(A.shape[0]):
                    torch._scaled_mm(A[b], B[b], scale_a=one, scale_b=one,
                                     out_dtype=torch.bfloat16, out=out[b])
                return out
            return torch._scaled_mm(A, B, scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                    out=out)
        return mm
    if device.type != "cuda" or w.backend == "torch":
        def mm(A, B, out):
            if A.dim() == 3:
                return torch.bmm(A, B, out=out)
            return torch.matmul(A, B, out=out)
        return mm
    if w.backend != "native":
        raise ValueError(f"unknown backend {w.backend!r}")
    kernel = w.kernel

    def mm(A, B, out):
        return _gemm.matmul(A, B, out=out, kernel=kernel)
    return mm


def kernel_label(w: Workload, A, B, out, shared: bool = False) -> str:
    """The kernel ``gemm_fn`` runs for this problem; ``shared``: as issued
    beside collectives (under ``ops.gemm.shared_device``, like the overlap
    schedules' GEMMs)."""
    if A.device.type != "cuda":
        return "torch.matmul(cpu)"
    if w.backend == "torch":
        return "torch._scaled_mm(hipBLASLt)" if w.dtype == _gemm.FP8 else "torch.matmul(hipBLASLt)"
    with (_gemm.shared_device() if shared else contextlib.nullcontext()):
        if w.kernel == "auto":
            padded = _gemm.padded_kernel_for(A, B, out)
            if padded:
                return f"{padded} (zero-padded K/N)"
        return _gemm.kernel_for(A, B, out, kernel=w.kernel)


def generator(device: torch.device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def randn(shape, w: Workload, device: torch.device, seed: int, operand: str = "A") -> torch.Tensor:
    """N(0,1) operands (random, non-zero data matters on MI355X: DVFS runs
    zero-filled GEMMs ~15-20% fast — cdna_hip_programming.md §5.4 rule 25).

    float8_e4m3fn: the N(0,1) draw rounded to e4m3 (well inside its ±448
    range, so the per-tensor scale is 1); a B operand (``operand="B"``) is
    laid out column-major, the fp8 kernel's B layout (same values)."""
    g = generator(device, seed)
    if w.dtype == _gemm.FP8:
        x = torch.randn(*shape, generator=g, device=device, dtype=torch.float32)
        if operand == "B":
            return x.transpose(-1, -2).contiguous().to(_gemm.FP8).transpose(-1, -2)
        return x.to(_gemm.FP8)
    return torch.randn(*shape, generator=g, device=device, dtype=w.dtype)


def out_dtype(w: Workload) -> torch.dtype:
    """dtype of the GEMM output C (bf16 for fp8 operands, else the operand dtype)."""
    return _gemm.out_dtype(w.dtype)


def zeros_b(rows: int, cols: int, w: Workload, device: torch.device) -> torch.Tensor:
    """A zeroed [rows, cols] B-operand buffer in the layout ``randn(..., operand="B")`` uses."""
    if w.dtype == _gemm.FP8:
        return torch.zeros((cols, rows), device=device, dtype=w.dtype).t()
    return torch.zeros((rows, cols), device=device, dtype=w.dtype)


def warmup(step: Callable[[], None], w: Workload, ctx: DistContext) -> None:
    """``w.warmup`` untimed steps, then — if ``w.min_warmup_ms`` is set — enough
    extra steps to reach that much warm-up time. MI355X clocks settle only after
    tens of ms of MFMA load (DVFS), so ten 0.1-ms GEMMs at 4k would leave the
    timed loop on a ramping clock. The extra count is agreed by a MAX all-reduce,
    so ranks running collectives in ``step`` stay in lock-step."""
    import math
    import time

    from ..parallel.dist import reduce_scalar

    for _ in range(w.warmup):
        step()
    if w.min_warmup_ms <= 0 or ctx.device.type != "cuda":
        return
    synchronize(ctx.device)
    t0 = time.perf_counter()
    step()
    synchronize(ctx.device)
    one = max((time.perf_counter() - t0) * 1e3, 1e-3)
    done_ms = one * (w.warmup + 1)
    extra = 0 if done_ms >= w.min_warmup_ms else min(10_000, math.ceil((w.min_warmup_ms - done_ms) / one))
    extra = int(reduce_scalar(ctx, float(extra), "max"))
    for _ in range(extra):
        step()


def align_ranks(ctx: DistContext) -> None:
    """Drain this rank's queue, then barrier (matmul_scaling_benchmark.py:78-82)."""
    synchronize(ctx.device)
    barrier(ctx)


def sampled_relerr(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, rows: int = 64,
                   seed: int = 1234) -> float:
    """Norm-relative error of ``C`` vs a float64 ``A @ B`` on ``rows`` sampled rows
    (all rows when M ≤ ``rows``). Replaces the dead, K-truncating
    ``validate_result`` of matmul_scaling_benchmark.py:240-249."""
    M = A.shape[-2]
    if M <= rows:
        idx = torch.arange(M, device=A.device)
    else:
        g = torch.Generator(device="cpu").manual_seed(seed)
        idx = torch.randperm(M, generator=g)[:rows].sort().values.to(A.device)
    Ar = A.index_select(-2, idx).double()
    ref = torch.matmul(Ar, B.double())
    got = C.index_select(-2, idx).double()
    den = ref.norm().clamp_min(1e-30)
    return float(((got - ref).norm() / den).item())


def validate_result(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor,
                    tol: Optional[float] = None) -> bool:
    """``C ≈ A @ B`` over the FULL reduction dimension (the reference's
    ``validate_result``, matmul_scaling_benchmark.py:240-249, truncates K to
    10 and is never called). Sampled rows, float64 reference, norm-relative
    tolerance of the dtype (``tolerance``) unless ``tol`` is given."""
    return sampled_relerr(A, B, C) < (tol if tol is not None else tolerance(C.dtype))


def allreduced_relerr(ctx: DistContext, A: torch.Tensor, B: torch.Tensor, C: torch.Tensor,
                      rows: int = 64, seed: int = 4321) -> float:
    """Check an all-reduced GEMM output: ``C`` must equal Σ_ranks A_r @ B_r.

    Every rank picks the same sampled rows, computes its own float64 partial
    product for them and the partials are SUM-all-reduced in float64, so the
    whole compute → (overlapped) collective path is verified without moving
    any operand between ranks. Collective: every rank must call it."""
    import torch.distributed as dist

    M = A.shape[-2]
    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = (torch.arange(M) if M <= rows else torch.randperm(M, generator=g)[:rows].sort().values)
    idx = idx.to(A.device)
    part = torch.matmul(A.index_select(-2, idx).double(), B.double())
    if ctx.is_distributed:
        dist.all_reduce(part)
    got = C.index_select(-2, idx).double()
    return float(((got - part).norm() / part.norm().clamp_min(1e-30)).item())


def tolerance(dtype: torch.dtype) -> float:
    """Norm-relative error budget of a fp32-accumulated GEMM with dtype outputs."""
    # fp8 operands: the reference is float64 of the SAME e4m3 values, so only the
    # bf16 output rounding remains.
    return {torch.bfloat16: 1e-2, torch.float16: 2e-3, torch.float32: 1e-5,
            _gemm.FP8: 1e-2}[dtype]
