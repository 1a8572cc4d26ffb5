"""FLOP / TFLOPS / efficiency formulas and the theoretical-peak table.

Reference parity:
  * ``calculate_tflops`` — matmul_benchmark.py:34-37 and
    matmul_scaling_benchmark.py:63-67 (``2·N³·num_ops / t / 1e12``).
  * peak table used for "GPU Efficiency" — matmul_benchmark.py:130-141
    (RTX 6000 Ada 182.2 / 91.1, Radeon RX 7900 XTX 123 / 61.4). The MI355X
    rows are the dense (non-sparse) figures of MI355X_MICROARCH.md:
    bf16/fp16 ≈2.5 PF, fp32 157.3 TF (exact-fp32 MFMA = vector rate; gfx950
    has no TF32).
  * Scaling efficiency — the reference's independent-mode number is
    SUM/(rank0·ws) (matmul_scaling_benchmark.py:315), i.e. rank imbalance,
    and the backup one is inverted (backup/matmul_distributed_benchmark.py:
    252-258). Here ``scaling_efficiency`` is the real thing:
    node throughput ÷ (ws × single-GPU throughput), and
    ``balance_efficiency`` keeps the reference's imbalance meaning under an
    honest name.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

DTYPES = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16,
          # MI355X extension: OCP e4m3 operands, bf16 output (ops/csrc/gemm_fp8.hip)
          "float8_e4m3fn": torch.float8_e4m3fn}
DTYPE_NAMES = {v: k for k, v in DTYPES.items()}


def dtype_from_name(name) -> torch.dtype:
    if isinstance(name, torch.dtype):
        return name
    try:
        return DTYPES[name]
    except KeyError:
        raise ValueError(f"unsupported dtype {name!r}; choose from {sorted(DTYPES)}") from None


def dtype_name(dt: torch.dtype) -> str:
    return DTYPE_NAMES.get(dt, str(dt))


def bytes_per_element(dt: torch.dtype) -> int:
    return torch.empty((), dtype=dt).element_size()


def gemm_flops(m: int, n: int, k: int, batch: int = 1) -> float:
    """FLOPs of ``batch`` GEMMs of shape [m,k]@[k,n] (one multiply + one add per MAC)."""
    return 2.0 * float(m) * float(n) * float(k) * float(batch)


def square_flops(n: int, num_ops: float = 1) -> float:
    return 2.0 * float(n) ** 3 * num_ops


def calculate_tflops(n: int, seconds: float, num_ops: float = 1) -> float:
    """TFLOPS of ``num_ops`` square N×N GEMMs done in ``seconds`` (0 if no time)."""
    if seconds <= 0:
        return 0.0
    return square_flops(n, num_ops) / seconds / 1e12


def tflops_from(flops: float, seconds: float) -> float:
    return flops / seconds / 1e12 if seconds > 0 else 0.0


@dataclass(frozen=True)
class Peak:
    gpu: str
    half: float  # bf16 / fp16 dense TFLOPS
    fp32: float
    fp8: Optional[float] = None  # e4m3 dense TFLOPS (None: not listed)

    def for_dtype(self, dt: torch.dtype) -> Optional[float]:
        if dt == torch.float8_e4m3fn:
            return self.fp8
        return self.fp32 if dt == torch.float32 else self.half


PEAKS = {
    # fp8 dense = 2x bf16 (block-scaled 16x16x128 / 32x32x64 MFMA, MI355X_MICROARCH.md)
    "mi355x": Peak("AMD Instinct MI355X", 2516.6, 157.3, 5033.2),
    "mi350x": Peak("AMD Instinct MI350X", 2306.9, 144.2, 4613.7),
    "rtx6000ada": Peak("RTX 6000 Ada", 182.2, 91.1),
    "rx7900xtx": Peak("Radeon RX 7900 XTX", 123.0, 61.4),
}


def peak_for_device(device_name: str, gcn_arch: Optional[str] = None) -> Optional[Peak]:
    """Theoretical peak for a device name (None if unknown — efficiency is then omitted).

    Unlike matmul_benchmark.py:131-139 (any "amd" name → 7900 XTX), an MI355X is
    recognised by name or by its gfx950 ISA.
    """
    n = (device_name or "").lower()
    arch = (gcn_arch or "").lower()
    if "mi355" in n or (arch.startswith("gfx950") and "mi350" not in n):
        return PEAKS["mi355x"]
    if "mi350" in n:
        return PEAKS["mi350x"]
    if "6000 ada" in n:
        return PEAKS["rtx6000ada"]
    if "7900" in n:
        return PEAKS["rx7900xtx"]
    return None


def percent_of_peak(tflops: float, peak: Optional[Peak], dt: torch.dtype) -> Optional[float]:
    if peak is None or not peak.for_dtype(dt):
        return None
    return 100.0 * tflops / peak.for_dtype(dt)


def scaling_efficiency(node_tflops: float, ws: int, single_gpu_tflops: float) -> Optional[float]:
    """Node throughput relative to ``ws`` × the measured 1-GPU throughput (percent)."""
    if single_gpu_tflops <= 0 or ws <= 0:
        return None
    return 100.0 * node_tflops / (ws * single_gpu_tflops)


def balance_efficiency(sum_tflops: float, rank0_tflops: float, ws: int) -> Optional[float]:
    """The reference's independent-mode "Scaling efficiency" (matmul_scaling_benchmark.py:315):
    SUM over ranks ÷ (rank-0 × ws). It measures rank imbalance, not scaling."""
    if rank0_tflops <= 0 or ws <= 0:
        return None
    return 100.0 * sum_tflops / (rank0_tflops * ws)


def overlap_efficiency(t_compute: float, t_total: float) -> Optional[float]:
    """Share of the step spent in compute (100% = communication fully hidden).

    Replaces the inverted backup formula (backup/matmul_distributed_benchmark.py:256-257)."""
    if t_total <= 0:
        return None
    return 100.0 * min(t_compute / t_total, 1.0)
