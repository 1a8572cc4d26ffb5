"""Process-group bring-up, collective self-test and cross-rank agreement.

Reference parity:
  * ``setup_distributed`` / ``cleanup_distributed`` — matmul_benchmark.py:9-32,
    matmul_scaling_benchmark.py:15-24,59-61.
  * ``verify_collectives`` — matmul_scaling_benchmark.py:26-57 (all_reduce of
    rank+1, all_gather of 2·rank, barrier), gated at :388-394.

MI355X-first differences:
  * GPU runs always use ``backend="nccl"``, which is RCCL on PyTorch-ROCm,
    over xGMI. The reference's "AMD device → gloo" switch
    (matmul_benchmark.py:14-21) would push every MI355X all-reduce through
    host TCP and is deliberately not reproduced (Q2). Gloo is used only for
    CPU tensors (``--device cpu`` and the CPU test-suite).
  * Device binding uses ``LOCAL_RANK`` (``rank % device_count`` is wrong as
    soon as there is more than one node), and the process group is bound
    to that device (``device_id=``) so RCCL communicators are created
    eagerly with the right device.
  * ``all_ok`` all-reduces a per-rank error flag so a failure on any rank
    (OOM, kernel error) makes every rank skip together instead of leaving
    the others blocked in the next collective.
  * ``reduce_scalar`` reduces metrics in float64 on the group's device.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None  # None: no process group (single process)

    @property
    def is_distributed(self) -> bool:
        return self.backend is not None and dist.is_available() and dist.is_initialized()

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def is_cuda(self) -> bool:
        return self.device.type == "cuda"


def env_world() -> tuple:
    """(rank, world_size, local_rank) from the torchrun environment (0, 1, 0 if absent)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        rank = int(os.environ["RANK"])
        ws = int(os.environ["WORLD_SIZE"])
        lr = int(os.environ.get("LOCAL_RANK", rank))
        return rank, ws, lr
    return 0, 1, 0


def resolve_device(device: str = "auto", local_rank: int = 0) -> torch.device:
    """``auto``: this rank's GPU if one is visible, else CPU."""
    if device in ("auto", None):
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("--device cuda requested but no GPU is visible")
        n = torch.cuda.device_count()
        # One rank per GPU in production. More ranks than GPUs (rank % n, as the
        # reference does) is only meaningful with the gloo backend, which lets a
        # single-GPU box rehearse the multi-rank GPU code paths; RCCL refuses two
        # ranks on one device.
        return torch.device("cuda", local_rank % n)
    if device == "cpu":
        return torch.device("cpu")
    return torch.device(device)


def setup_distributed(device: str = "auto", timeout_s: float = 600.0,
                      backend: Optional[str] = None) -> DistContext:
    """Initialise from torchrun env vars; single-process context if they are absent."""
    rank, ws, lr = env_world()
    dev = resolve_device(device, lr)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ctx = DistContext(rank=rank, world_size=ws, local_rank=lr, device=dev, backend=None)
    if ws <= 1 and "RANK" not in os.environ:
        return ctx
    if not dist.is_initialized():
        be = backend or ("nccl" if dev.type == "cuda" else "gloo")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(**kw)
        ctx.backend = be
    else:
        ctx.backend = dist.get_backend()
    ctx.rank = dist.get_rank()
    ctx.world_size = dist.get_world_size()
    return ctx


def cleanup_distributed() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier(ctx: DistContext) -> None:
    if not ctx.is_distributed:
        return
    if ctx.backend == "nccl" and ctx.is_cuda:
        dist.barrier(device_ids=[ctx.device.index])
    else:
        dist.barrier()


def _scalar(ctx: DistContext, value: float) -> torch.Tensor:
    return torch.tensor([float(value)], dtype=torch.float64, device=ctx.device)


def reduce_scalar(ctx: DistContext, value: float, op: str = "sum") -> float:
    """All-reduce one float across ranks (``sum`` | ``avg`` | ``max`` | ``min``)."""
    if not ctx.is_distributed:
        return float(value)
    t = _scalar(ctx, value)
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
           "avg": dist.ReduceOp.SUM}
    dist.all_reduce(t, op=ops[op])
    v = float(t.item())
    return v / ctx.world_size if op == "avg" else v


def gather_scalars(ctx: DistContext, value: float) -> List[float]:
    """Every rank's value, in rank order (on every rank)."""
    if not ctx.is_distributed:
        return [float(value)]
    t = _scalar(ctx, value)
    out = torch.empty(ctx.world_size, dtype=torch.float64, device=ctx.device)
    dist.all_gather_into_tensor(out, t)
    return [float(x) for x in out.tolist()]


def all_ok(ctx: DistContext, ok: bool) -> bool:
    """True iff ``ok`` holds on every rank (collective; every rank must call it)."""
    if not ctx.is_distributed:
        return bool(ok)
    return reduce_scalar(ctx, 0.0 if ok else 1.0, "sum") == 0.0


def verify_collectives(ctx: DistContext, verbose: bool = True) -> bool:
    """Runtime self-test of the collectives the benchmark relies on.

    all_reduce(SUM) of rank+1 must equal ws(ws+1)/2; all_gather_into_tensor of
    2·rank must return 0,2,4,…; a large bf16 all_reduce must be exact for
    small integers (exercises the RCCL bulk path, not just the 4-byte one);
    then a barrier. Returns False on any mismatch or exception (on all ranks).
    """
    ok = True
    try:
        ws = ctx.world_size
        t = _scalar(ctx, ctx.rank + 1.0)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        ok &= abs(t.item() - ws * (ws + 1) / 2.0) < 1e-9
        g = torch.empty(ws, dtype=torch.float64, device=ctx.device)
        dist.all_gather_into_tensor(g, _scalar(ctx, 2.0 * ctx.rank))
        ok &= all(abs(v - 2.0 * i) < 1e-9 for i, v in enumerate(g.tolist()))
        big = torch.full((1 << 20,), float(ctx.rank + 1), dtype=torch.bfloat16, device=ctx.device)
        dist.all_reduce(big)
        ok &= bool((big.float() == ws * (ws + 1) / 2.0).all().item())
        barrier(ctx)
    except Exception as e:  # pragma: no cover - only on broken fabrics
        print(f"[rank {ctx.rank}] collective self-test raised: {e!r}", flush=True)
        ok = False
    try:
        ok = all_ok(ctx, ok)
    except Exception:  # pragma: no cover
        ok = False
    if ok and verbose and ctx.is_main:
        print(f"✓ Collective operations verified successfully across {ctx.world_size} GPUs"
              if ctx.is_cuda else
              f"✓ Collective operations verified successfully across {ctx.world_size} processes",
              flush=True)
    return ok
