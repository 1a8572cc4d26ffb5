#!/usr/bin/env python3
"""Driver benchmark: whole-node TFLOPS of the 16k×16k bf16 GEMM on N MI355X GPUs.

Metric and config are BASELINE.json's headline: "TFLOPS (whole node) +
scaling efficiency, 16k×16k bf16 GEMM at 1/2/4/8 GPUs" — the reference's
``matmul_benchmark.py`` / ``matmul_scaling_benchmark.py --mode independent``
16384² bf16 number (README.md:43-44: ~140 TFLOPS on 1 RTX 6000 Ada, ~294 on 2).

One "step" = one 16384×16384×16384 bf16 GEMM per GPU on the hand-written
gfx950 MFMA kernel (``--mode independent``, weak scaling: per-GPU work is
fixed as N grows). ``--mode batch_parallel`` (bmm + RCCL all-reduce of the
output) and ``--mode matrix_parallel`` (column-sharded B + RCCL all-gather,
strong scaling) are available too. W untimed warmup steps, then exactly K
timed steps bracketed by barrier + synchronize on both sides; the max over
ranks of the elapsed wall time is the step time; rank 0 prints one JSON line.

After the headline measurement (which is what ``value`` reports) the same
process also times the reference's other two scaling modes — batch_parallel
(matmul_scaling_benchmark.py:106-165) and matrix_parallel (:167-238), each
serialized as in the reference and with the collective overlapped on the
comm stream — for ``--extra-steps`` steps each, and reports them under
``"modes"`` in the same JSON line, so one launch at N GPUs yields the
BASELINE configs 3-5 (``--extra-steps 0`` skips them).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without torchrun self-launches N ranks (a child
``torch.distributed.run``, started before anything touches the GPU) and exits
with its code; under torchrun, ``WORLD_SIZE != --gpus`` is an error. At N > 1
the job also times the headline GEMM on rank 0 alone (others at a barrier)
and reports ``scaling_efficiency = value / (N x single_gpu_tflops)`` — the
1 -> N curve's efficiency from one launch. Every mode's setup is agreed
across ranks (a setup failure becomes an ``"error"`` entry, no hang); a
failure inside a timed region exits that rank at once, so torchrun tears the
job down in seconds (fault injection: ``PDMB_BENCH_FAULT=rank:mode:phase``).
"""
from __future__ import annotations

import argparse
import contextlib
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import (  # noqa: E402
    BidirRing, GatherOverlap, ReduceOverlap, all_gather_now, compute_ctx, compute_stream, gemm_chunks)
from pytorch_distributed_matmul_benchmark_amd.parallel.comm import CommStream  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.dist import (  # noqa: E402
    DistContext, all_ok, barrier, cleanup_distributed, reduce_scalar, setup_distributed)
from pytorch_distributed_matmul_benchmark_amd.parallel.partition import (  # noqa: E402
    column_shard, global_batch, local_batch)

# Reference numbers (README.md:43-46): whole-system TFLOPS at 16k bf16.
BASELINE_TFLOPS = {"independent": {1: 140.0, 2: 294.0},
                   "batch_parallel": {1: 140.0, 2: 237.0},
                   "matrix_parallel": {1: 140.0, 2: 141.0}}
METRIC = "TFLOPS (whole node) + scaling efficiency, 16k×16k bf16 GEMM at 1/2/4/8 GPUs"
DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
          "float8_e4m3fn": torch.float8_e4m3fn}


class Workload:
    """Operands + one timed ``step()`` of a scaling mode on this rank."""

    def __init__(self, a, ctx, mode: str, overlap: bool):
        self.ctx, self.mode, self.overlap = ctx, mode, overlap
        self.cuda = ctx.device.type == "cuda"
        self.dt = DTYPES[a.dtype]
        self.backend = a.backend
        dev, n, ws, dt = ctx.device, a.size, ctx.world_size, self.dt
        odt = gemm.out_dtype(dt)  # fp8 operands write a bf16 C
        self._g = torch.Generator(device=dev)
        flop_gemm = 2.0 * n * n * n
        overlap = overlap and ws > 1
        comp = torch.cuda.current_stream(dev) if self.cuda else None
        self._mask = None
        if overlap and self.cuda and a.comm_cus > 0:
            # GEMM chunks on a CU-masked stream, RCCL gets the free CUs at once
            comp, self._mask = compute_stream(dev, a.comm_cus)
        self.comp = comp

        if mode == "independent":
            A, B = self._rnd(n, n, seed=2 * ctx.rank), self._rnd(n, n, seed=2 * ctx.rank + 1, b=True)
            C = torch.empty(n, n, device=dev, dtype=odt)
            self.kernel = self._label(A, B, C)

            def step():
                self._mm(A, B, C)
            self.flops = flop_gemm * ws
            self.global_batch, self.parallelism = ws, f"independent{ws}"
        elif mode == "batch_parallel":
            lb, gb = local_batch(ws), global_batch(ws)
            A = self._rnd(lb, n, n, seed=2 * ctx.rank)
            B = self._rnd(lb, n, n, seed=2 * ctx.rank + 1, b=True)
            C = torch.empty(lb, n, n, device=dev, dtype=odt)
            self.kernel = self._label(A, B, C)
            if overlap:
                ov = ReduceOverlap(lb, gemm_chunks(n, n, a.chunks, dt, dev), dev)
                _, s0, e0 = ov.units[0]  # what a chunk runs beside the reductions
                self.kernel = self._label(A[0, s0:e0], B[0], C[0, s0:e0], shared=True)

                def step():
                    with compute_ctx(self.comp, self._mask):
                        ov.step(self._mm, A, B, C, self.comp)
                    self._join()
            else:
                def step():
                    self._mm(A, B, C)
                    if ws > 1:
                        dist.all_reduce(C)
            self.flops = flop_gemm * gb
            self.global_batch, self.parallelism = gb, f"dp{ws}"
        elif mode == "matrix_parallel":
            sh = column_shard(n, ws, ctx.rank, align=8)
            A = self._rnd(n, n, seed=10_000)
            Bg = self._rnd(n, n, seed=10_001, b=True)
            Bl = (torch.zeros(sh.padded, n, device=dev, dtype=dt).t() if dt == gemm.FP8
                  else torch.zeros(n, sh.padded, device=dev, dtype=dt))
            Bl[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
            del Bg
            Cl = torch.empty(n, sh.padded, device=dev, dtype=odt)
            self.kernel = self._label(A, Bl, Cl)
            if overlap:
                ov = GatherOverlap(n, sh.padded, ws, dev, odt,
                                   gemm_chunks(n, sh.padded, a.chunks, dt, dev),
                                   pieces=a.comm_chunks, requested=a.chunks, impl=a.allgather)
                s0, e0 = ov.chunks[0]  # what a chunk runs beside the gathers
                self.kernel = self._label(A[s0:e0], Bl, Cl[s0:e0], shared=True)

                def step():
                    with compute_ctx(self.comp, self._mask):
                        ov.step(self._mm, A, Bl, Cl, self.comp)
                    self._join()
            else:
                gathered = torch.empty(ws * n, sh.padded, device=dev, dtype=odt)
                cs = CommStream(dev) if a.allgather == "direct" else None

                def step():
                    self._mm(A, Bl, Cl)
                    if ws > 1:
                        all_gather_now(gathered, Cl, a.allgather, cs)
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"tp{ws}"
        elif mode == "ring_parallel":
            # Opt-in (not timed by default): all-gather-GEMM over both ring
            # directions, models/ring_parallel.py. A half-blocks rotate by P2P
            # behind each hop's GEMMs.
            rs, sh = column_shard(n, ws, ctx.rank, align=512), column_shard(n, ws, ctx.rank, align=8)
            A = self._rnd(n, n, seed=10_000)
            Al = torch.zeros(rs.padded, n, device=dev, dtype=dt)
            Al[:rs.width].copy_(A[rs.start:rs.stop])
            del A
            Bg = self._rnd(n, n, seed=10_001, b=True)
            Bl = (torch.zeros(sh.padded, n, device=dev, dtype=dt).t() if dt == gemm.FP8
                  else torch.zeros(n, sh.padded, device=dev, dtype=dt))
            Bl[:, :sh.width].copy_(Bg[:, sh.start:sh.stop])
            del Bg
            rp = rs.padded
            Cl = torch.empty(ws * rp, sh.padded, device=dev, dtype=odt)
            self.kernel = self._label(Al[:rp // 2], Bl, Cl[:rp // 2], shared=True)
            ring = BidirRing(Al, rp, ctx.rank, ws, dev)

            def step():
                with gemm.shared_device():  # the hops' transfers run beside these GEMMs
                    ring.step(self._mm, Bl, Cl, self.comp)
            self.flops = flop_gemm
            self.global_batch, self.parallelism = 1, f"ring{ws}"
        else:
            raise ValueError(mode)
        self.step = step

    def _rnd(self, *shape, seed, b=False):
        """N(0,1) operand; fp8: rounded to e4m3 (scale 1), a B operand column-major."""
        self._g.manual_seed(seed)
        if self.dt != gemm.FP8:
            return torch.randn(*shape, generator=self._g, device=self.ctx.device, dtype=self.dt)
        x = torch.randn(*shape, generator=self._g, device=self.ctx.device, dtype=torch.float32)
        if b:
            return x.transpose(-1, -2).contiguous().to(gemm.FP8).transpose(-1, -2)
        return x.to(gemm.FP8)

    def _mm(self, A, B, out):
        if self.dt == gemm.FP8 and self.cuda and self.backend == "torch":
            one = torch.ones((), device=A.device)
            return torch._scaled_mm(A, B, scale_a=one, scale_b=one, out_dtype=torch.bfloat16,
                                    out=out)
        if (self.backend == "torch" or not self.cuda) and self.dt != gemm.FP8:
            return torch.matmul(A, B, out=out)
        return gemm.matmul(A, B, out=out)

    def _join(self):
        """The timing (current) stream waits for the masked compute stream."""
        if self._mask is not None:
            torch.cuda.current_stream(self.ctx.device).wait_stream(self.comp)

    def _label(self, A, B, C, shared=False):
        """The kernel the step's GEMMs run (shared: beside collectives, as
        compute_ctx / the ring issue them, under gemm.shared_device)."""
        if not self.cuda:
            return "torch.matmul(cpu)"
        if self.backend != "native":
            return "hipBLASLt"
        with (gemm.shared_device() if shared else contextlib.nullcontext()):
            return gemm.kernel_for(A, B, C)

    def _sync(self):
        if self.cuda:
            torch.cuda.synchronize(self.ctx.device)

    def timed(self, warmup: int, steps: int) -> float:
        """W untimed steps, then K steps bracketed by sync+barrier; max-over-ranks seconds."""
        for _ in range(warmup):
            self.step()
        self._sync()
        barrier(self.ctx)
        self._sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        self._sync()
        barrier(self.ctx)
        self._sync()
        elapsed = time.perf_counter() - t0
        if self.ctx.is_distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.ctx.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed


def _free(ctx) -> None:
    gc.collect()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)
        torch.cuda.empty_cache()


def _self_launch(a) -> int:
    """``--gpus N > 1`` outside torchrun: start N ranks as a child
    ``torch.distributed.run`` (the reference's launcher pattern,
    run_scaling_benchmark.sh:23-31) and exit with its code. Nothing here has
    touched the GPU (``import torch`` does not initialise HIP), so the child
    ranks own their devices from scratch; the parent only waits."""
    import subprocess

    if a.device == "cuda" and a.dist_backend in ("auto", "nccl"):
        ndev = torch.cuda.device_count()  # does not initialise HIP on this image
        if ndev < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but only {ndev} GPU(s) visible; RCCL needs one GPU "
                  f"per rank (use --dist-backend gloo to rehearse more ranks than GPUs)",
                  file=sys.stderr, flush=True)
            return 2
    # no --master-port: --standalone binds port 0 itself (a port picked here
    # could be taken by another process before the child listens on it)
    where = ([f"--master-addr=127.0.0.1", f"--master-port={a.master_port}"] if a.master_port
             else ["--standalone", "--local-addr=127.0.0.1"])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", *where, os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, PDMB_BENCH_CHILD="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def _fault(ctx, key: str, phase: str) -> None:
    """Fault injection for the failure-agreement tests: ``PDMB_BENCH_FAULT=
    rank:mode:phase`` (mode ``*`` = any; phase ``setup`` | ``timed``) raises
    on that rank at that point."""
    spec = os.environ.get("PDMB_BENCH_FAULT")
    if not spec:
        return
    r, m, p = spec.split(":")
    if int(r) == ctx.rank and m in (key, "*") and p == phase:
        raise RuntimeError(f"injected fault (rank {ctx.rank}, {key}, {phase})")


def _die(ctx, key: str, exc: BaseException) -> None:
    """A failure inside a timed region cannot be agreed on (the other ranks are
    already blocked in a collective this rank will never join): report it and
    exit at once, so torchrun's agent tears the job down in seconds instead of
    every peer waiting out the process-group timeout."""
    import traceback

    print(f"[rank {ctx.rank}] {key} failed in the timed region: {exc!r}", file=sys.stderr,
          flush=True)
    traceback.print_exc(file=sys.stderr)
    sys.stderr.flush()
    sys.stdout.flush()
    os._exit(1)


def _measure(a, ctx, mode: str, overlap: bool, warmup: int, steps: int, key: str):
    """Build (agreed across ranks) and time one workload. Returns
    ``(tflops, seconds, workload_info)`` or ``(None, None, error_string)``."""
    w, err = None, None
    try:
        _fault(ctx, key, "setup")
        w = Workload(a, ctx, mode, overlap)
    except Exception as e:  # OOM, unsupported shape, ...: every rank skips together
        err = f"{type(e).__name__}: {e}"
        print(f"[rank {ctx.rank}] {key} setup failed: {err}", file=sys.stderr, flush=True)
    if not all_ok(ctx, err is None):
        del w
        _free(ctx)
        return None, None, err or "failed on another rank"
    try:
        _fault(ctx, key, "timed")
        el = w.timed(warmup, steps)
    except Exception as e:
        _die(ctx, key, e)
    v = w.flops * steps / el / 1e12 if el > 0 else 0.0
    info = dict(global_batch=w.global_batch, parallelism=w.parallelism, kernel=w.kernel)
    del w
    _free(ctx)
    return v, el, info


def _single_gpu_tflops(a, ctx):
    """The '1 GPU' denominator of the scaling efficiency: the headline GEMM
    timed on rank 0 alone (same K/W, same device) while every other rank
    waits at a barrier — measured in the same job, so the 1 -> N curve needs
    no second launch. The reference's own "Scaling efficiency" is rank
    imbalance, not scaling (matmul_scaling_benchmark.py:315)."""
    val = 0.0
    barrier(ctx)
    if ctx.rank == 0:
        try:
            one = DistContext(rank=0, world_size=1, local_rank=ctx.local_rank, device=ctx.device)
            w = Workload(a, one, "independent", False)
            el = w.timed(a.warmup, a.steps)
            val = w.flops * a.steps / el / 1e12 if el > 0 else 0.0
            del w
        except Exception as e:  # a failed reference is "no efficiency", never a hang
            print(f"[rank 0] single-GPU reference failed: {e!r}", file=sys.stderr, flush=True)
            val = 0.0
        _free(ctx)
    barrier(ctx)
    v = reduce_scalar(ctx, val, "sum")
    return v if v > 0 else None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--dtype", default="bfloat16", choices=list(DTYPES))
    ap.add_argument("--mode", default="independent",
                    choices=["independent", "batch_parallel", "matrix_parallel", "ring_parallel"])
    ap.add_argument("--overlap", action="store_true",
                    help="batch/matrix_parallel: hide the collective behind the GEMM chunks")
    ap.add_argument("--chunks", type=int, default=4,
                    help="overlap: GEMM row chunks (capped so each chunk fills the chip)")
    ap.add_argument("--comm-chunks", type=int, default=0,
                    help="matrix_parallel --overlap: all-gather pieces per GEMM chunk "
                         "(0: enough pieces for --chunks in total)")
    ap.add_argument("--comm-cus", type=int, default=0,
                    help="overlap: CUs kept free of GEMM workgroups for RCCL (CU-masked "
                         "compute stream; 0 = no mask)")
    ap.add_argument("--allgather", default="rccl", choices=["rccl", "direct"],
                    help="matrix_parallel all-gather: RCCL, or direct P2P to every peer at once")
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: torch.matmul + gloo, to exercise the multi-rank path without a GPU")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--master-port", type=int, default=0,
                    help="self-launch rendezvous port (0: a free one)")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="timed steps for each secondary mode reported under \"modes\" "
                         "(batch_parallel / matrix_parallel, serialized and overlapped); 0: skip")
    ap.add_argument("--extra-warmup", type=int, default=3)
    ap.add_argument("--no-scaling-ref", action="store_true",
                    help="N > 1: skip the in-job 1-GPU reference (scaling_efficiency = null)")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            return _self_launch(a)
    elif int(os.environ["WORLD_SIZE"]) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}",
              file=sys.stderr, flush=True)
        return 2

    ctx = setup_distributed(a.device, timeout_s=float(os.environ.get("PDMB_PG_TIMEOUT", "300")),
                            backend=None if a.dist_backend == "auto" else a.dist_backend)
    cuda = ctx.device.type == "cuda"
    ws = ctx.world_size
    dt = DTYPES[a.dtype]
    headline16k = dt == torch.bfloat16 and a.size == 16384 and cuda

    def vs_base(mode, value):
        base = BASELINE_TFLOPS.get(mode, {}).get(ws) if headline16k else None
        return round(value / base, 3) if base and value is not None else None

    # Headline: the metric BASELINE.json names, measured first on a quiet node.
    value, elapsed, head = _measure(a, ctx, a.mode, a.overlap, a.warmup, a.steps, a.mode)
    if value is None:
        if ctx.is_main:
            print(f"bench.py: headline {a.mode} failed: {head}", file=sys.stderr, flush=True)
        cleanup_distributed()
        return 1
    ms_step = elapsed / max(a.steps, 1) * 1e3

    single = value if ws == 1 and a.mode == "independent" else None
    if ws > 1 and not a.no_scaling_ref:
        single = _single_gpu_tflops(a, ctx)

    def eff(v):
        return round(v / (ws * single), 4) if single and v is not None else None

    # Secondary modes (BASELINE configs 4-5): same operands' shapes and dtype, own timing.
    # At ws = 1 there is no collective to overlap: those entries are null, not a
    # second copy of the serialized number.
    modes = {}
    if a.extra_steps > 0:
        for mode, ov in (("batch_parallel", False), ("batch_parallel", True),
                         ("matrix_parallel", False), ("matrix_parallel", True)):
            if mode == a.mode and ov == a.overlap:
                continue
            key = mode + ("+overlap" if ov else "")
            if ov and ws == 1:
                modes[key] = None
                continue
            v, el, info = _measure(a, ctx, mode, ov, a.extra_warmup, a.extra_steps, key)
            if v is None:
                modes[key] = {"error": info}
                continue
            modes[key] = {"value": round(v, 4), "ms_per_step": round(el / a.extra_steps * 1e3, 4),
                          "steps": a.extra_steps, "warmup": a.extra_warmup,
                          "global_batch": info["global_batch"], "parallelism": info["parallelism"],
                          "scaling": "strong" if mode == "matrix_parallel" else "weak",
                          "vs_baseline": vs_base(mode, v), "scaling_efficiency": eff(v),
                          "kernel": info["kernel"]}

    if ctx.is_main:
        out = {
            "metric": METRIC, "value": round(value, 4), "unit": "TFLOPS",
            "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if a.mode in ("matrix_parallel", "ring_parallel") else "weak",
            "vs_baseline": vs_base(a.mode, value),
            "scaling_efficiency": eff(value),
            "single_gpu_tflops": round(single, 4) if single else None,
            "dtype": {"bfloat16": "bf16", "float16": "fp16", "float32": "fp32",
                      "float8_e4m3fn": "fp8_e4m3"}[a.dtype],
            "data": "synthetic (torch.randn N(0,1) operands, seeded per rank)",
            "device": ctx.device.type,
            "config": {"model": f"gemm_{a.size}x{a.size}x{a.size}_{a.dtype}",
                       "global_batch": head["global_batch"], "seq_len": a.size,
                       "parallelism": head["parallelism"], "mode": a.mode,
                       "overlap": bool(a.overlap), "backend": a.backend, "kernel": head["kernel"]},
            "per_gpu_tflops": (round(value / ws, 2)
                               if a.mode not in ("matrix_parallel", "ring_parallel") else None),
            "vs_reference_1gpu_linear": round(value / (140.0 * ws), 3),
            "modes": modes,
        }
        print(json.dumps(out), flush=True)
    cleanup_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
