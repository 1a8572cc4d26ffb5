"""Probe (next-round input): would the wave-quantisation tail pay for fp8 W4?
fp8 W4 over whole-wave rows + an S-way split fp8 W4 launch for the tail rows, vs
auto (one launch) and hipBLASLt _scaled_mm. One JSON line per (shape, variant)."""
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
    f8 = torch.float8_e4m3fn
    for M, N, K in [(6144, 6144, 6144), (6000, 6000, 6144), (7168, 7168, 7168), (10240, 10240, 10240)]:
        torch.manual_seed(0)
        A = (torch.randn(M, K, device="cuda") * 0.5).to(f8)
        Bt = (torch.randn(N, K, device="cuda") * 0.5).to(f8)
        B = Bt.t()  # column-major K x N
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        one = torch.ones((), device="cuda")
        res = {"auto": timeit(lambda: gemm.matmul(A, B, out=C)),
               "torch": timeit(lambda: torch._scaled_mm(A, B, one, one, out_dtype=torch.bfloat16))}
        tm, tn = (M + 255) // 256, (N + 255) // 256
        for rows in range(1, tm):
            M1 = (tm - rows) * 256
            if M1 * 0 + (tm - rows) * tn > 2 * 256 + 256 or rows * tn * 2 > 256:
                continue
            def two():
                gemm.matmul(A[:M1], B, out=C[:M1], kernel="fp8_w4", splitk=1)
                gemm.matmul(A[M1:], B, out=C[M1:], kernel="fp8_w4", splitk=2)
            try:
                res[f"tail{rows}xS2"] = timeit(two)
            except RuntimeError as e:
                print(json.dumps({"M": M, "rows": rows, "err": str(e)[:80]}), flush=True)
        fl = 2.0 * M * N * K
        for k, v in res.items():
            print(json.dumps({"M": M, "N": N, "K": K, "variant": k, "us": round(v, 1),
                              "tflops": round(fl / v / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
