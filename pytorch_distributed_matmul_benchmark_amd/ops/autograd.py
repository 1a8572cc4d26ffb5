"""``native_matmul``: the gfx950 MFMA GEMM as a differentiable op.

Forward ``C = A @ B`` and both backward GEMMs (``dA = dC @ Bᵀ``,
``dB = Aᵀ @ dC``) run on the native kernels; transposed operands are
materialised row-major first (the kernels take row-major NN operands with a
unit inner stride). Lets the benchmark GEMM drop into a training step
(used by ``__graft_entry__.smoke``).
"""
from __future__ import annotations

import torch

from . import gemm


class _NativeMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, B):
        ctx.save_for_backward(A, B)
        return gemm.matmul(A, B)

    @staticmethod
    def backward(ctx, dC):
        A, B = ctx.saved_tensors
        dC = dC.contiguous()
        dA = dB = None
        if ctx.needs_input_grad[0]:
            dA = gemm.matmul(dC, B.transpose(-1, -2).contiguous())
            if A.dim() == 2 and dA.dim() == 3:  # A broadcast over B's batch
                dA = dA.sum(0)
        if ctx.needs_input_grad[1]:
            if A.dim() == 3:
                dB = gemm.matmul(A.transpose(-1, -2).contiguous(), dC)
                if B.dim() == 2:
                    dB = dB.sum(0)
            else:
                dB = gemm.matmul(A.transpose(-1, -2).contiguous(), dC)
        return dA, dB


def native_matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    return _NativeMatmul.apply(A, B)
