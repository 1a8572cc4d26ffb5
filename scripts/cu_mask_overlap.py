#!/usr/bin/env python3
"""CU budget for communication: what a CU-masked GEMM stream buys an overlapped
collective, measured on ONE GPU with a comm proxy.

RCCL's collectives are CU kernels. Next to a GEMM that holds every CU with one
256-thread workgroup for a whole K-loop (W4 at 16k: ~300 us per workgroup),
a collective kernel launched mid-GEMM — even on a high-priority stream — gets
CUs only as GEMM workgroups retire. ``--comm-cus k`` (parallel/overlap.py
MaskedStream) runs the GEMM on a stream whose CU mask excludes k CUs (spread
over the 8 XCDs), so the collective starts at once on those.

Arms (interleaved rounds, best of each):
  gemm_k        the GEMM alone on a stream masked by k CUs (k = 0: no mask)
  proxy         the comm proxy alone on the high-priority stream
  both_k        GEMM (masked by k) and the proxy issued together, the proxy on
                the high-priority stream behind an event recorded after the
                GEMM's first chunk — the overlap schedule's shape
hidden_k = (gemm_k + proxy - both_k) / proxy: the fraction of the proxy's
time hidden behind the GEMM (1 = fully hidden, 0 = serialized).

The proxy is an elementwise ``torch.add`` of two bf16 buffers into a third
(RCCL's reduce-copy inner loop is the same HBM-bound shape), sized like a
matrix_parallel all-gather piece.

    python scripts/cu_mask_overlap.py [--n 16384] [--chunks 4] [--proxy-mib 64]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.comm import new_stream  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import MaskedStream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--shard", type=int, default=2048, help="GEMM N (a ws=8 column shard)")
    ap.add_argument("--chunks", type=int, default=4, help="GEMM row chunks per step")
    ap.add_argument("--proxy-mib", type=float, default=64.0, help="bytes per proxy operand")
    ap.add_argument("--cus", type=int, nargs="+", default=[0, 8, 16, 32])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    n, sh = a.n, a.shard
    A = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(n, sh, device=dev, dtype=torch.bfloat16)
    C = torch.empty(n, sh, device=dev, dtype=torch.bfloat16)
    rows = n // a.chunks
    el = int(a.proxy_mib * (1 << 20) / 2)
    x = torch.randn(el, device=dev, dtype=torch.bfloat16)
    y = torch.randn(el, device=dev, dtype=torch.bfloat16)
    z = torch.empty_like(x)
    comm = new_stream(dev, high_priority=True)
    masked = {k: (MaskedStream(dev, k) if k > 0 else None) for k in a.cus}
    for k, ms in masked.items():
        if ms is not None:
            print(json.dumps({"cus_excluded": k, "active_cus": ms.active_cus()}), flush=True)

    def gemm_step(stream, ev=None, proxy=False):
        with torch.cuda.stream(stream):
            for j in range(a.chunks):
                gemm.matmul(A[j * rows:(j + 1) * rows], B, out=C[j * rows:(j + 1) * rows])
                if proxy:
                    ev[j].record(stream)
                    comm.wait_event(ev[j])
                    with torch.cuda.stream(comm):
                        torch.add(x, y, out=z)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            fn()
        torch.cuda.current_stream().wait_stream(comm)
        for ms in masked.values():
            if ms is not None:
                torch.cuda.current_stream().wait_stream(ms.stream)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    cur = torch.cuda.current_stream()
    evs = [torch.cuda.Event() for _ in range(a.chunks)]
    best = {}

    def keep(name, ms):
        best[name] = min(best.get(name, float("inf")), ms)

    for _ in range(3):  # warm-up (clocks, allocator, counters)
        gemm_step(cur)
    for _ in range(a.rounds):
        keep("proxy", timed(lambda: [torch.add(x, y, out=z) for _ in range(a.chunks)]))
        for k, ms in masked.items():
            st = ms.stream if ms is not None else cur
            keep(f"gemm_{k}", timed(lambda: gemm_step(st)))
            keep(f"both_{k}", timed(lambda: gemm_step(st, evs, proxy=True)))
    flops = 2.0 * n * n * sh
    for k in a.cus:
        g, p, b = best[f"gemm_{k}"], best["proxy"], best[f"both_{k}"]
        print(json.dumps({
            "cus_excluded": k, "gemm_ms": round(g, 4), "gemm_tflops": round(flops / g / 1e9, 1),
            "proxy_ms": round(p, 4), "both_ms": round(b, 4),
            "hidden": round((g + p - b) / p, 3) if p > 0 else None,
            "n": n, "shard": sh, "chunks": a.chunks, "proxy_mib": a.proxy_mib,
            "kernel": gemm.kernel_for(A[:rows], B)}), flush=True)
    for ms in masked.values():
        if ms is not None:
            ms.close()


if __name__ == "__main__":
    main()
