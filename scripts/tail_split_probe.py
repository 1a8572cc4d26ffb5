"""Probe: W4 over the whole waves of 256-row tile stripes + a split-K launch for
the remaining stripes, vs one W4 launch, on grids whose last wave is partly
empty. Prints one JSON line per (shape, variant)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    ts = []
    for _ in range(rounds):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    shapes = [(6000, 6000, 6144), (5000, 5000, 5056), (3000, 7000, 5056), (6144, 6144, 6144),
              (10000, 10000, 10048)]
    for M, N, K in shapes:
        torch.manual_seed(0)
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        R = torch.matmul(A, B)
        fl = 2.0 * M * N * K
        tm, tn = (M + 255) // 256, (N + 255) // 256
        res = {"auto": timeit(lambda: gemm.matmul(A, B, out=C)),
               "torch": timeit(lambda: torch.matmul(A, B, out=R))}
        for rows in range(1, tm):  # tail stripes (tile rows) split over K
            M1 = (tm - rows) * 256
            for S in (2, 3, 4):
                def two():
                    gemm.matmul(A[:M1], B, out=C[:M1], kernel="w4", splitk=1)
                    gemm.matmul(A[M1:], B, out=C[M1:], kernel="w4", splitk=S)
                if rows * tn * S > 256 or (K // 64) // S < 4:
                    continue
                try:
                    res[f"tail{rows}xS{S}"] = timeit(two)
                except RuntimeError as e:
                    t = torch.empty(M - M1, K, device="cuda", dtype=torch.bfloat16)
                    try:
                        gemm.matmul(t, B, kernel="w4", splitk=S)
                        fresh = "ok"
                    except RuntimeError as e2:
                        fresh = str(e2)[:60]
                    print(json.dumps({"M": M, "tail_rows": M - M1, "S": S, "err": str(e)[:60],
                                      "fresh_tensor": fresh}), flush=True)
        best = min((v, k) for k, v in res.items() if k.startswith("tail")) if len(res) > 2 else None
        err = (C.float() - R.float()).norm() / R.float().norm()
        for k, v in res.items():
            print(json.dumps({"M": M, "N": N, "K": K, "variant": k, "us": round(v, 1),
                              "tflops": round(fl / v / 1e6, 1)}), flush=True)
        print(json.dumps({"M": M, "N": N, "K": K, "best_tail": best, "relerr_last": err.item()}), flush=True)


if __name__ == "__main__":
    main()
