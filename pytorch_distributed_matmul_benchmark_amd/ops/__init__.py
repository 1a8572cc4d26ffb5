"""Compute ops: hand-written gfx950 MFMA GEMM kernels (``csrc/``) + bindings."""
from .gemm import bench_matmul, bmm, kernel_for, matmul  # noqa: F401
