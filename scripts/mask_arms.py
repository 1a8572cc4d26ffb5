#!/usr/bin/env python3
"""The 16k GEMM on a CU-masked stream (parallel/overlap.py MaskedStream, k CUs
left out, spread over the XCDs): which kernel the planner picks under the
budget, and how the dispatch-balanced W4 compares with the persistent W4S
sized to the budget (G = 256 - k workgroups). Interleaved rounds, median ms.

    python scripts/mask_arms.py [--n 16384] [--cus 0 8 16 32] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import MaskedStream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--ncols", type=int, default=0, help="GEMM N (0: n)")
    ap.add_argument("--cus", type=int, nargs="+", default=[0, 8, 16, 32])
    ap.add_argument("--kernels", default="auto,w4,w4s")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, nc = a.n, a.ncols or a.n
    torch.manual_seed(0)
    A = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(n, nc, device=dev, dtype=torch.bfloat16)
    C = torch.empty(n, nc, device=dev, dtype=torch.bfloat16)
    R = gemm.matmul(A, B, kernel="w4")
    flops = 2.0 * n * n * nc
    arms, streams = [], {}
    for k in a.cus:
        ms = MaskedStream(dev, k) if k > 0 else None
        streams[k] = ms
        for kern in a.kernels.split(","):
            arms.append((k, kern))

    def run(k, kern, iters):
        ms = streams[k]
        st = ms.stream if ms else torch.cuda.current_stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st), gemm.cu_budget(ms.cus if ms else 0):
            e0.record(st)
            for _ in range(iters):
                gemm.matmul(A, B, out=C, kernel=kern)
            e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    res, label = {}, {}
    for k, kern in arms:
        ms = streams[k]
        with gemm.cu_budget(ms.cus if ms else 0):
            label[(k, kern)] = gemm.kernel_for(A, B, C, kernel=kern)
        run(k, kern, 2)
        ok = torch.equal(C, R) if kern != "auto" else bool(((C.float() - R.float()).abs().max()) < 1)
        res[(k, kern)] = {"times": [], "ok": ok}
    for r in range(a.rounds):
        for arm in (arms if r % 2 == 0 else arms[::-1]):
            res[arm]["times"].append(run(*arm, a.iters))
    for (k, kern), v in res.items():
        t = statistics.median(v["times"])
        print(json.dumps({"m": n, "n": nc, "k": n, "comm_cus": k, "kernel": kern,
                          "resolved": label[(k, kern)], "median_ms": round(t, 4),
                          "tflops": round(flops / t / 1e9, 1), "ok": v["ok"]}), flush=True)
    for ms in streams.values():
        if ms:
            ms.close()


if __name__ == "__main__":
    main()
