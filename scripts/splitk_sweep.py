#!/usr/bin/env python3
"""Under-filled-grid GEMMs: W4 / T128 x split-K (and auto) vs hipBLASLt, interleaved.

Shapes default to the per-rank matrix_parallel shards of the reference's default
sizes (matmul_scaling_benchmark.py:179-188 at :351-352) plus 2048^3. Both arms
are timed as hipGraph replays of ``--iters`` launches (native: bench_matmul
graph=True; hipBLASLt: torch.cuda.graph of torch.matmul), so host launch
overhead is out of the comparison for the ~20-120 us problems. Rounds are
interleaved (DVFS), the best round per arm is reported, one JSON line per
(shape, arm).

    python scripts/splitk_sweep.py [--shapes 8192x1024x8192 ...] [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

SHAPES = ["8192x1024x8192", "4096x512x4096", "2048x2048x2048", "4096x1024x4096",
          "8192x2048x8192", "16384x2048x16384", "4096x2048x4096", "16384x16384x16384"]


def torch_graph_ms(A, B, out, iters):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.matmul(A, B, out=out)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            torch.matmul(A, B, out=out)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=SHAPES)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-ms", type=float, default=20.0, help="GPU time per timed graph")
    ap.add_argument("--arms", nargs="+",
                    default=["auto", "w4:1", "w4:2", "t128:1", "t128:2", "t128:4"],
                    help="kernel:splitk (auto = the dispatcher's plan)")
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    for shp in a.shapes:
        m, n, k = (int(x) for x in shp.lower().split("x"))
        torch.manual_seed(0)
        A = torch.randn(m, k, device="cuda", dtype=dt)
        B = torch.randn(k, n, device="cuda", dtype=dt)
        out = torch.empty(m, n, device="cuda", dtype=dt)
        R = torch.matmul(A.float(), B.float())
        flops = 2.0 * m * n * k
        iters = max(5, int(a.min_ms * 1e-3 / (flops / 1.0e15)))  # ~min_ms at 1 PF
        arms = {}
        tiles = (m // 256) * (n // 256)
        for arm in a.arms:
            kern, _, sk = arm.partition(":")
            S = int(sk or 0)
            if S > 1 and tiles > 1024:
                continue  # a full grid: split-K only adds partial traffic
            try:
                name = gemm.kernel_for(A, B, kernel=kern)
                real = gemm.splitk_for(A, B, kernel=kern, splitk=S)
                gemm.matmul(A, B, out=out, kernel=kern, splitk=S)
            except Exception as e:  # noqa: BLE001 (S not valid for this K / shape)
                print(json.dumps({"shape": shp, "arm": arm, "skipped": str(e)[:120]}), flush=True)
                continue
            err = ((out.float() - R).norm() / R.norm()).item()
            arms[arm] = dict(kernel=kern, S=S, name=name, real=real, err=err)
        arms["hipblaslt"] = dict()
        best = {k_: float("inf") for k_ in arms}
        for _ in range(a.rounds):
            for name, info in arms.items():
                if name == "hipblaslt":
                    ms = torch_graph_ms(A, B, out, iters)
                else:
                    ms = gemm.bench_matmul(A, B, out, iters=iters, warmup=2, graph=True,
                                           kernel=info["kernel"], splitk=info["S"])
                best[name] = min(best[name], ms / iters)
        for name, info in arms.items():
            rec = {"shape": shp, "arm": name, "us": round(best[name] * 1e3, 2),
                   "tflops": round(flops / (best[name] * 1e-3) / 1e12, 1), "iters": iters,
                   "rounds": a.rounds, "dtype": a.dtype}
            if name != "hipblaslt":
                rec.update(kernel=info["name"], splitk_requested=info["S"], splitk=info["real"],
                           relerr=round(info["err"], 6))
            print(json.dumps(rec), flush=True)
        del A, B, out, R
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
