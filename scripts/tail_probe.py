#!/usr/bin/env python3
"""Wave-quantisation tail and batch-launch probe, one process, interleaved rounds.

Tail (--shapes M,N,K): auto (the planner's plan), hipBLASLt, and every forced
two-launch plan "tail{r}xS{S}": rows [0, M1) as one unsplit launch (W4S / fp8
W4S where that launch has >= 2 tiles per CU, else W4 / fp8 W4), then the last
r tile rows as one S-way split-K launch. Shows whether gemm_dispatch.cpp
tail_plan's model leaves a measured win on the table (10240^3 fp8: 6.25 waves).

Batch (--batch B, with one square --shapes entry): bmm of B on one launch vs B
single launches of the same GEMM back to back ("seq"), the two ways
batch_parallel can run its local work.

    python scripts/tail_probe.py --dtype float8_e4m3fn --shapes 10240,10240,10240 6144,6144,6144
    python scripts/tail_probe.py --dtype bfloat16 --shapes 16384,16384,16384 --batch 4
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float8_e4m3fn")
    ap.add_argument("--shapes", nargs="+", default=["10240,10240,10240"])
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--max-rows", type=int, default=4, help="largest tail in tile rows")
    ap.add_argument("--arms", default="", help="comma list: keep only these arms")
    ap.add_argument("--trace", type=int, default=0,
                    help="no timing: run each arm N times, synchronized, in order (under "
                         "rocprofv3 --kernel-trace; prints the arm order)")
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    fp8 = dt == torch.float8_e4m3fn
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    one = torch.ones((), device="cuda")
    for s in a.shapes:
        M, N, K = (int(v) for v in s.split(","))
        torch.manual_seed(0)
        lead = (a.batch,) if a.batch else ()
        if fp8:
            A, _ = gemm.fp8_quantize(torch.randn(*lead, M, K, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(*lead, K, N, device="cuda"), colmajor=True)
        else:
            A = torch.randn(*lead, M, K, device="cuda", dtype=dt)
            B = torch.randn(*lead, K, N, device="cuda", dtype=dt)
        C = torch.empty(*lead, M, N, device="cuda", dtype=gemm.out_dtype(dt))
        flops = 2.0 * M * N * K * max(a.batch, 1)

        def vendor():
            if fp8 and a.batch:  # _scaled_mm takes matrices only
                for b in range(a.batch):
                    torch._scaled_mm(A[b], B[b], one, one, out_dtype=torch.bfloat16, out=C[b])
            elif fp8:
                torch._scaled_mm(A, B, one, one, out_dtype=torch.bfloat16, out=C)
            else:
                torch.matmul(A, B, out=C)

        arms = {"auto": lambda: gemm.matmul(A, B, out=C), "torch": vendor}
        if a.batch:
            def seq():
                for b in range(a.batch):
                    gemm.matmul(A[b], B[b], out=C[b])
            arms["seq"] = seq
            one_launch = "fp8_w4s" if fp8 else "w4s"
            arms["one_launch"] = lambda: gemm.matmul(A, B, out=C, kernel=one_launch)
        else:
            tm, tn = (M + 255) // 256, (N + 255) // 256
            whole, split = ("fp8_w4s", "fp8_w4") if fp8 else ("w4s", "w4")
            for r in range(1, min(a.max_rows, tm - 1) + 1):
                M1 = (tm - r) * 256
                first = whole if (tm - r) * tn >= 2 * cus and (K // (128 if fp8 else 64)) % 2 == 0 else split
                for S in (2, 3, 4):
                    if r * tn * S > cus:
                        continue

                    def two(M1=M1, first=first, S=S):
                        gemm.matmul(A[:M1], B, out=C[:M1], kernel=first, splitk=0 if first.endswith("s") else 1)
                        gemm.matmul(A[M1:], B, out=C[M1:], kernel=split, splitk=S)
                    try:
                        two()
                        torch.cuda.synchronize()
                    except RuntimeError as e:
                        print(json.dumps({"shape": s, "arm": f"tail{r}xS{S}", "err": str(e)[:100]}), flush=True)
                        continue
                    arms[f"tail{r}xS{S}"] = two
        if a.arms:
            arms = {k: f for k, f in arms.items() if k in a.arms.split(",")}
        if a.trace:
            for k, f in arms.items():
                for _ in range(a.trace):
                    f()
                torch.cuda.synchronize()
                print(json.dumps({"shape": s, "trace_arm": k, "launches": a.trace}), flush=True)
            continue
        R = torch.matmul(A.float(), B.float()) if not fp8 else None
        for name, f in list(arms.items()):  # every arm computes the same C
            f()
            torch.cuda.synchronize()
            if R is not None and name != "torch":
                err = ((C.float() - R).norm() / R.norm()).item()
                if err > 1e-2:
                    print(json.dumps({"shape": s, "arm": name, "bad_relerr": err}), flush=True)
                    del arms[name]
        del R
        res = {k: [] for k in arms}
        for _ in range(2):
            for f in arms.values():
                timed(f, 3)
        for _ in range(a.rounds):
            for k, f in arms.items():
                res[k].append(timed(f, a.iters))
        plan = gemm.tail_split_for(A, B) if not a.batch else None
        best = min(res, key=lambda k: statistics.median(res[k]))
        for k in arms:
            med = statistics.median(res[k])
            print(json.dumps({"shape": s, "dtype": a.dtype, "batch": a.batch, "arm": k,
                              "median_us": round(med, 1), "tflops": round(flops / med / 1e6, 1),
                              "min_us": round(min(res[k]), 1), "auto_kernel": gemm.kernel_for(A, B),
                              "auto_tail": plan, "best": best}), flush=True)
        del A, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
