"""Reference-compatible function API.

The reference exposes its building blocks as module-level functions with these
exact signatures; code written against them can import this module instead.
Every function runs on this package's engine (gfx950 MFMA kernels, RCCL,
event-ordered comm streams) and keeps the reference's return conventions
(times in SECONDS, TFLOPS as the reference defines them per mode).

  matmul_benchmark.py:9-79            setup_distributed, cleanup_distributed,
                                      calculate_tflops, benchmark_matmul
  matmul_scaling_benchmark.py:10-249  ScalingMode, verify_collectives,
                                      benchmark_independent, benchmark_batch_parallel,
                                      benchmark_matrix_parallel, validate_result
  backup/matmul_distributed_benchmark.py:35-174
                                      benchmark_independent_backup (the 3-tuple
                                      variant), benchmark_data_parallel,
                                      benchmark_model_parallel
  backup/matmul_overlap_benchmark.py:36-278
                                      benchmark_no_overlap, benchmark_overlap,
                                      benchmark_pipeline (pipeline_depth)
  MI355X addition (no reference counterpart)
                                      benchmark_ring_parallel (all-gather-GEMM
                                      over the ring, models/ring_parallel.py)
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist

from .models import BenchmarkMode, ScalingMode  # noqa: F401  (re-exported)
from .models import batch_parallel as _bp
from .models import data_parallel as _dp
from .models import independent as _ind
from .models import matrix_parallel as _mp
from .models import model_parallel as _mdp
from .models import overlap as _ov
from .models import ring_parallel as _rp
from .models.common import Workload
from .models.common import validate_result as _validate
from .parallel import dist as _dist
from .utils.metrics import calculate_tflops  # noqa: F401  (same formula and signature)


def setup_distributed() -> Tuple[int, int]:
    """``(rank, world_size)``; initialises RCCL from the torchrun env if present
    (matmul_scaling_benchmark.py:15-24)."""
    ctx = _dist.setup_distributed("auto")
    return ctx.rank, ctx.world_size


def cleanup_distributed() -> None:
    _dist.cleanup_distributed()


def _ctx(device, rank=None, world_size=None) -> _dist.DistContext:
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if dist.is_available() and dist.is_initialized():
        return _dist.DistContext(rank=dist.get_rank(), world_size=dist.get_world_size(),
                                 local_rank=dev.index or 0, device=dev,
                                 backend=dist.get_backend())
    return _dist.DistContext(rank=rank or 0, world_size=1, local_rank=dev.index or 0, device=dev)


def _w(matrix_size, dtype, iters, warmup, **kw) -> Workload:
    return Workload(n=int(matrix_size), dtype=dtype, iters=int(iters), warmup=int(warmup), **kw)


def verify_collectives(rank: int, world_size: int, device: str) -> bool:
    return _dist.verify_collectives(_ctx(device, rank, world_size))


def benchmark_matmul(matrix_size: int, dtype: torch.dtype, device: str, num_iterations: int = 50,
                     warmup_iterations: int = 10) -> Tuple[float, float]:
    """(avg seconds per GEMM, TFLOPS) — matmul_benchmark.py:39-79."""
    r = _ind.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device))
    return r.avg_ms / 1e3, r.tflops


def benchmark_independent(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                          num_iterations: int = 50, warmup_iterations: int = 10
                          ) -> Tuple[float, float]:
    """matmul_scaling_benchmark.py:69-104 (per-rank seed, barrier after warm-up)."""
    r = _ind.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device, rank))
    return r.avg_ms / 1e3, r.tflops


def benchmark_batch_parallel(matrix_size: int, batch_size: int, dtype: torch.dtype, device: str,
                             rank: int, world_size: int, num_iterations: int = 50,
                             warmup_iterations: int = 10) -> Tuple[float, float]:
    """matmul_scaling_benchmark.py:106-165; the batch is never split to zero."""
    r = _bp.run(_w(matrix_size, dtype, num_iterations, warmup_iterations, batch=batch_size),
                _ctx(device, rank, world_size))
    return r.avg_ms / 1e3, r.tflops


def benchmark_matrix_parallel(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                              world_size: int, num_iterations: int = 50,
                              warmup_iterations: int = 10) -> Tuple[float, float]:
    """matmul_scaling_benchmark.py:167-238 (TFLOPS = 2N³ / t / ws)."""
    r = _mp.run(_w(matrix_size, dtype, num_iterations, warmup_iterations),
                _ctx(device, rank, world_size))
    return r.avg_ms / 1e3, r.tflops


def validate_result(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, tolerance: float = 1e-3
                    ) -> bool:
    """Full-K check (the reference's truncates K to 10); ``tolerance`` is a
    norm-relative bound, raised to the dtype's rounding floor for 16-bit outputs."""
    from .models.common import tolerance as _tol

    return _validate(A, B, C, max(tolerance, _tol(C.dtype)))


def _backup(r) -> Tuple[float, float, float]:
    return r.avg_ms / 1e3, r.tflops, (r.comm_ms or 0.0) / 1e3


def benchmark_independent_backup(matrix_size: int, dtype: torch.dtype, device: str,
                                 num_iterations: int = 50, warmup_iterations: int = 10
                                 ) -> Tuple[float, float, float]:
    """backup/matmul_distributed_benchmark.py:35-64 → (t, tflops, 0.0)."""
    r = _ind.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device))
    return r.avg_ms / 1e3, r.tflops, 0.0


def benchmark_data_parallel(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                            num_iterations: int = 50, warmup_iterations: int = 10
                            ) -> Tuple[float, float, float]:
    """backup/matmul_distributed_benchmark.py:66-110 → (t_total, compute TFLOPS, t_comm)."""
    return _backup(_dp.run(_w(matrix_size, dtype, num_iterations, warmup_iterations),
                           _ctx(device, rank)))


def benchmark_model_parallel(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                             world_size: int, num_iterations: int = 50,
                             warmup_iterations: int = 10) -> Tuple[float, float, float]:
    """backup/matmul_distributed_benchmark.py:112-174, shape bug fixed."""
    return _backup(_mdp.run(_w(matrix_size, dtype, num_iterations, warmup_iterations),
                            _ctx(device, rank, world_size)))


def benchmark_no_overlap(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                         num_iterations: int = 50, warmup_iterations: int = 10
                         ) -> Tuple[float, float, float]:
    """backup/matmul_overlap_benchmark.py:36-91 → (t/iter, compute-only TFLOPS, t_comm)."""
    r = _ov.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device, rank),
                mode="no_overlap")
    return r.avg_ms / 1e3, r.compute_only_tflops or 0.0, (r.comm_ms or 0.0) / 1e3


def benchmark_overlap(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                      num_iterations: int = 50, warmup_iterations: int = 10
                      ) -> Tuple[float, float, float]:
    """backup/matmul_overlap_benchmark.py:93-180, event-ordered."""
    r = _ov.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device, rank),
                mode="overlap")
    return r.avg_ms / 1e3, r.compute_only_tflops or 0.0, (r.comm_ms or 0.0) / 1e3


def benchmark_ring_parallel(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                            world_size: int, num_iterations: int = 50,
                            warmup_iterations: int = 10) -> Tuple[float, float]:
    """Ring all-gather-GEMM, same return convention as benchmark_matrix_parallel
    (seconds, TFLOPS = 2N³ / t / ws)."""
    r = _rp.run(_w(matrix_size, dtype, num_iterations, warmup_iterations),
                _ctx(device, rank, world_size))
    return r.avg_ms / 1e3, r.tflops


def benchmark_pipeline(matrix_size: int, dtype: torch.dtype, device: str, rank: int,
                       num_iterations: int = 50, warmup_iterations: int = 10,
                       pipeline_depth: int = 3) -> Tuple[float, float, float]:
    """backup/matmul_overlap_benchmark.py:182-278 (ring of ``pipeline_depth`` buffers)."""
    r = _ov.run(_w(matrix_size, dtype, num_iterations, warmup_iterations), _ctx(device, rank),
                mode="pipeline", depth=pipeline_depth)
    return r.avg_ms / 1e3, r.compute_only_tflops or 0.0, (r.comm_ms or 0.0) / 1e3
