#!/usr/bin/env python3
"""Host cost per GEMM call: a Python loop of ``gemm.matmul`` on tiny and small
problems (GPU time negligible or known), against ``torch.matmul`` and the
planner alone (``plan_shape``). One JSON line per case: microseconds per call
(wall clock over N calls, synchronized at the end).

    python scripts/host_overhead.py [--calls 2000]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import _native, gemm  # noqa: E402


def per_call(fn, calls):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / calls * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    C = _native.load(build_if_missing=False)
    for n, dt in ((256, torch.bfloat16), (1024, torch.bfloat16), (2048, torch.bfloat16), (1024, torch.float32)):
        A = torch.randn(n, n, device="cuda", dtype=dt)
        B = torch.randn(n, n, device="cuda", dtype=dt)
        out = torch.empty(n, n, device="cuda", dtype=dt)
        code = {torch.bfloat16: 2, torch.float32: 0}[dt]
        rec = {"n": n, "dtype": str(dt).split(".")[-1],
               "native_us": round(per_call(lambda: gemm.matmul(A, B, out=out), a.calls), 2),
               "torch_us": round(per_call(lambda: torch.matmul(A, B, out=out), a.calls), 2),
               "plan_shape_us": round(per_call(lambda: C.plan_shape(code, n, n, n, 1, 0, 0), a.calls), 2),
               "gpu_us": round(gemm.bench_matmul(A, B, out, 200, 20) / 200 * 1e3, 2)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
