#!/usr/bin/env python3
"""In-kernel stamp diagnostic of the default GEMM schedule (SCHED 2).

Runs the native kernel back-to-back for ~2 s (steady clock), then one launch
of the stamp build, which records per wave the cycles spent waiting in the
barrier that closes each read slot (wr) and each compute slot (wc), plus the
K-loop's total cycles. Read SHARES, not absolute length (the stamps fence the
schedule). Prints a JSON summary.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import _native, gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--warm-s", type=float, default=2.0)
    a = ap.parse_args()
    n = a.n
    torch.manual_seed(0)
    A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    ref = gemm.matmul(A, B)
    t0 = time.time()
    while time.time() - t0 < a.warm_s:
        for _ in range(10):
            gemm.matmul(A, B, out=C)
        torch.cuda.synchronize()
    blocks = ((n + 255) // 256) ** 2
    dbg = torch.zeros(blocks * 8 * 4, dtype=torch.int64, device="cuda")
    mod = _native.load()
    mod.set_debug_buffer(dbg)
    try:
        gemm.matmul(A, B, out=C, kernel="mfma256c_stamp")
        torch.cuda.synchronize()
    finally:
        mod.set_debug_buffer(None)
    ok = torch.equal(C, ref)
    d = dbg.view(blocks, 8, 4).double()
    wr, wc, tot, nk = d[..., 0], d[..., 1], d[..., 2], d[..., 3]
    slots = nk * 8  # 4 phases x 2 slots per K-tile
    out = {"n": n, "stamp_output_equal_to_default": ok}
    for name, sl in (("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
        out[name] = {
            "wait_after_read_slot_share": float((wr[:, sl] / tot[:, sl]).mean()),
            "wait_after_compute_slot_share": float((wc[:, sl] / tot[:, sl]).mean()),
            "cycles_per_slot": float((tot[:, sl] / slots[:, sl]).mean()),
            "cycles_per_slot_p10_p90": [float(x) for x in torch.quantile(
                (tot[:, sl] / slots[:, sl]).flatten(), torch.tensor([0.1, 0.9], dtype=torch.float64,
                                                                      device="cuda"))],
        }
    out["ideal_cycles_per_slot"] = 256  # 16 MFMA 16x16x32 x 16 cycles per wave
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
