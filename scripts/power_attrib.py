#!/usr/bin/env python3
"""Where the 16k bf16 GEMM's power goes (VERDICT r4 "Next round" #8).

At 16k the chip is power-bound: W4S runs 83.9 % MFMA busy at 1.725 GHz
(profiles/r6c_pmc_w4s_16k.md) while a loop of nothing but v_mfma_f32_16x16x32
on random bf16 reaches 2055 TF (profiles/r2_mfma_shape_probe.jsonl). Which of
the kernel's other energy consumers holds the clock down? Timing-only W4S
variants (PDMB_EXPERIMENTS=1 build; WRONG results) each drop one:

  w4s                  the shipping kernel
  diag_w4s_nofrag      no LDS fragment reads (MFMAs re-use their registers)
  diag_w4s_nodma       no LDS-DMA refills (HBM / L2 / LDS-write traffic)
  diag_w4s_noepi       no C stores (the epilogue's LDS round trip + HBM writes)
  diag_w4s_mfma_only   neither reads nor refills: MFMAs, waits and barriers

Each arm runs back to back for ``--seconds`` per round (interleaved rounds,
rotating order) under the 5 ms amdsmi sampler: TFLOPS, median GFX clock,
median socket power, and TFLOPS per GHz (the work per clock — what the
MFMA-issue schedule sustains independent of the clock). One JSON line per arm
with the medians over rounds.

    PDMB_EXPERIMENTS=1 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench
    python scripts/power_attrib.py [--n 16384] [--rounds 3] [--seconds 2]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.utils.telemetry import ClockSampler  # noqa: E402

ARMS = ["w4s", "diag_w4s_nofrag", "diag_w4s_nodma", "diag_w4s_noepi", "diag_w4s_mfma_only"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--arms", default=",".join(ARMS))
    a = ap.parse_args()
    arms = a.arms.split(",")
    dev = torch.device("cuda", 0)
    n = a.n
    torch.manual_seed(0)
    A = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    B = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    C = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * n ** 3
    # launches per timed burst, from one launch of the shipping kernel
    one = gemm.bench_matmul(A, B, C, 3, 1, kernel="w4s") / 3
    iters = max(3, int(a.seconds * 1e3 / one))
    res = {k: {"tflops": [], "sclk_mhz": [], "power_w": []} for k in arms}
    for k in arms:  # warm every arm (and the clocks)
        gemm.bench_matmul(A, B, C, 5, 1, kernel=k)
    for r in range(a.rounds):
        for k in arms[r % len(arms):] + arms[:r % len(arms)]:
            torch.cuda.synchronize()
            with ClockSampler(dev) as smp:
                ms = gemm.bench_matmul(A, B, C, iters, 2, kernel=k)
            t = smp.result()
            res[k]["tflops"].append(flops * iters / (ms / 1e3) / 1e12)
            res[k]["sclk_mhz"].append(t["sclk_mhz"] or 0.0)
            res[k]["power_w"].append(t["power_w"] or 0.0)
            time.sleep(0.2)
    base = None
    for k in arms:
        tf = statistics.median(res[k]["tflops"])
        clk = statistics.median(res[k]["sclk_mhz"])
        pw = statistics.median(res[k]["power_w"])
        rec = {"n": n, "kernel": k, "iters": iters, "rounds": a.rounds, "tflops": round(tf, 1),
               "sclk_mhz": round(clk, 1), "power_w": round(pw, 1),
               "tflops_per_ghz": round(tf / (clk / 1e3), 1) if clk else None,
               "tflops_rounds": [round(x, 1) for x in res[k]["tflops"]]}
        if base is None:
            base = rec
        else:
            rec["vs_w4s"] = {"tflops": round(tf / base["tflops"], 4),
                             "sclk": round(clk / base["sclk_mhz"], 4) if base["sclk_mhz"] else None,
                             "power": round(pw / base["power_w"], 4) if base["power_w"] else None}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
