#!/usr/bin/env python3
"""CU budget for communication: what a CU-masked GEMM stream buys an overlapped
collective, measured on ONE GPU with a comm proxy.

RCCL's collectives are CU kernels. Next to a GEMM that holds every CU with one
256-thread workgroup for a whole K-loop (W4 at 16k: ~300 us per workgroup),
a collective kernel launched mid-GEMM — even on a high-priority stream — gets
CUs only as GEMM workgroups retire. ``--comm-cus k`` (parallel/overlap.py
MaskedStream) runs the GEMM on a stream whose CU mask excludes k CUs (spread
over the 8 XCDs), so the collective starts at once on those.

Arms (interleaved rounds, best of each), per (k, proxy size):
  gemm_k        the chunked GEMM alone on a stream masked by k CUs (k = 0: no
                mask), planned for the CUs it may use (ops.gemm.cu_budget)
  proxy         the comm proxy alone on the high-priority comm stream
  both_k        GEMM chunk j (masked by k), then proxy piece j on the comm
                stream behind an event recorded after it — round 2's chunked
                overlap schedule (profiles/r2_cu_mask_overlap_v*.jsonl: the
                chunked GEMM lost more than the overlap hid; round 3 replaced
                it with parallel/overlap.py OverlapPipeline, measured by
                scripts/overlap_proxy.py)
speedup_k = (gemm_0 + proxy) / both_k: the gain over running the same work
serialized without a mask (1 = nothing hidden, 2 = perfect overlap of equals).

The proxy (ops.gemm.comm_proxy) is a 16-B copy with a fixed number of
256-thread workgroups (--proxy-blocks, default 32): an RCCL collective's CU
footprint (a few tens of channels), HBM-bound like its reduce-copy loop.
Two proxy sizes: a compute-bound step (proxy < GEMM) and a comm-bound one.

    python scripts/cu_mask_overlap.py [--n 16384] [--chunks 4] [--proxy-mib 16 256]
"""
import argparse
import contextlib
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
    ap.add_argument("--proxy-mib", type=float, nargs="+", default=[16.0, 256.0],
                    help="bytes copied per chunk by the proxy")
    ap.add_argument("--proxy-blocks", type=int, default=32)
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
    comm = new_stream(dev, high_priority=True)
    masked = {k: (MaskedStream(dev, k) if k > 0 else None) for k in a.cus}
    plans = {}
    for k, ms in masked.items():
        with (ms.budget() if ms is not None else contextlib.nullcontext()):
            plans[k] = (gemm.kernel_for(A[:rows], B), gemm.splitk_for(A[:rows], B))
        if ms is not None:
            print(json.dumps({"cus_excluded": k, "active_cus": ms.active_cus(),
                              "chunk_plan": plans[k]}), flush=True)
    cur = torch.cuda.current_stream()
    evs = [torch.cuda.Event() for _ in range(a.chunks)]

    def run(k, proxy_bufs, do_gemm=True, do_proxy=True):
        ms = masked[k]
        st = ms.stream if ms is not None else cur
        ctx = ms.budget() if ms is not None else contextlib.nullcontext()
        st.wait_stream(cur)
        comm.wait_stream(cur)
        with torch.cuda.stream(st), ctx:
            for j in range(a.chunks):
                if do_gemm:
                    gemm.matmul(A[j * rows:(j + 1) * rows], B, out=C[j * rows:(j + 1) * rows])
                if do_proxy:
                    evs[j].record(st)
                    comm.wait_event(evs[j])
                    with torch.cuda.stream(comm):
                        gemm.comm_proxy(proxy_bufs[1], proxy_bufs[0], a.proxy_blocks)
        cur.wait_stream(st)
        cur.wait_stream(comm)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    flops = 2.0 * n * n * sh
    for mib in a.proxy_mib:
        el = int(mib * (1 << 20) / 2)
        bufs = (torch.randn(el, device=dev, dtype=torch.bfloat16),
                torch.empty(el, device=dev, dtype=torch.bfloat16))
        for _ in range(2):  # warm-up (clocks, allocator, split-K counters per stream)
            for k in a.cus:
                run(k, bufs)
        best = {}
        for _ in range(a.rounds):
            best["proxy"] = min(best.get("proxy", 1e9), timed(lambda: run(0, bufs, do_gemm=False)))
            for k in a.cus:
                best[f"gemm_{k}"] = min(best.get(f"gemm_{k}", 1e9),
                                        timed(lambda: run(k, bufs, do_proxy=False)))
                best[f"both_{k}"] = min(best.get(f"both_{k}", 1e9), timed(lambda: run(k, bufs)))
        g0, p = best["gemm_0"], best["proxy"]
        for k in a.cus:
            g, b = best[f"gemm_{k}"], best[f"both_{k}"]
            print(json.dumps({
                "cus_excluded": k, "proxy_mib_per_chunk": mib, "proxy_blocks": a.proxy_blocks,
                "gemm_ms": round(g, 4), "gemm_tflops": round(flops / g / 1e9, 1),
                "proxy_ms": round(p, 4), "both_ms": round(b, 4),
                "serial_unmasked_ms": round(g0 + p, 4), "speedup_vs_serial": round((g0 + p) / b, 3),
                "n": n, "shard": sh, "chunks": a.chunks, "chunk_plan": plans[k]}), flush=True)
        del bufs
    for ms in masked.values():
        if ms is not None:
            ms.close()


if __name__ == "__main__":
    main()
