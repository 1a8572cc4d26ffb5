#!/usr/bin/env python3
"""Tile timeline of the 256x256 kernels (W4 bf16, W4 fp8): where a workgroup's
time goes outside the K-loop, measured in-kernel (experiment build:
PDMB_EXPERIMENTS=1; trace ids diag_w4_trace / diag_fp8_w4_trace).

Each workgroup stamps s_memrealtime (chip-wide 100 MHz) at start, when the
first K-tile's fragments are in registers, at the end of the K-loop and after
its C stores drained, plus its CU (HW_ID) and XCC (ops/csrc/common.h
tile_trace_write). Per (kernel, shape) this prints, in microseconds:

  prologue / loop / epilogue   per-workgroup medians (and p90)
  gap                          per CU, start of a tile minus the end of the
                               CU's previous tile (dispatch + launch cost)
  loop_frac                    sum of K-loop time over all CUs / (CUs x span):
                               the fraction of the kernel the CUs spend in
                               their K-loops (the rest is fixed per-tile cost
                               and tail)
  tail                         last tile end minus the median CU's last end

    python scripts/tile_timeline.py --kernels w4 --shapes 16384,16384,1024 16384,16384,16384
    python scripts/tile_timeline.py --kernels fp8_w4 --dtype float8_e4m3fn --shapes ...
    python scripts/tile_timeline.py --kernels w4s ...   # W4S: one row per workgroup
                                                       # (start, end), so loop / epilogue read 0
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def cu_key(hw: int, xcc: int):
    return (xcc & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 0x1, (hw >> 8) & 0xF)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def analyse(tr: torch.Tensor) -> dict:
    rows = [r for r in tr.tolist() if r[0] != 0]
    t0 = min(r[0] for r in rows)
    span = max(r[3] for r in rows) - t0
    pro = [r[1] - r[0] for r in rows]
    loop = [r[2] - r[1] for r in rows]
    epi = [r[3] - r[2] for r in rows]
    per_cu = {}
    for r in rows:
        per_cu.setdefault(cu_key(r[4], r[5]), []).append(r)
    gaps, ends, loop_sum = [], [], 0
    for wgs in per_cu.values():
        wgs.sort(key=lambda r: r[0])
        for a, b in zip(wgs, wgs[1:]):
            gaps.append(b[0] - a[3])
        ends.append(wgs[-1][3])
        loop_sum += sum(r[2] - r[1] for r in wgs)
    first_starts = sorted(min(r[0] for r in w) for w in per_cu.values())
    per_xcd = {}
    for r in rows:
        per_xcd.setdefault(r[5] & 0xF, []).append(r[3])
    xcd_end = {x: statistics.median(v) - t0 for x, v in sorted(per_xcd.items())}
    per_xcd_loop, per_xcd_start = {}, {}
    for r in rows:
        per_xcd_loop.setdefault(r[5] & 0xF, []).append(r[2] - r[1])
        per_xcd_start.setdefault(r[5] & 0xF, []).append(r[1] - t0)

    def us(x):
        return round(x * TICK_US, 2)

    return {
        "workgroups": len(rows), "cus": len(per_cu), "span_us": us(span),
        "prologue_us": us(statistics.median(pro)), "prologue_p90_us": us(pct(pro, 0.9)),
        "loop_us": us(statistics.median(loop)),
        "epilogue_us": us(statistics.median(epi)), "epilogue_p90_us": us(pct(epi, 0.9)),
        "gap_us": us(statistics.median(gaps)) if gaps else None,
        "gap_p90_us": us(pct(gaps, 0.9)) if gaps else None,
        "first_start_spread_us": us(first_starts[-1] - first_starts[0]),
        "loop_frac": round(loop_sum / (len(per_cu) * span), 4),
        "tail_us": us(max(ends) - statistics.median(ends)),
        # median end of each XCD's workgroups: XCDs that run faster idle at the end
        "xcd_end_us": [us(v) for v in xcd_end.values()],
        # per XCD: median K-loop time and median time its K-loops started
        "xcd_loop_us": [us(statistics.median(v)) for _, v in sorted(per_xcd_loop.items())],
        "xcd_loop_start_us": [us(statistics.median(v)) for _, v in sorted(per_xcd_start.items())],
        "loop_min_us": us(min(loop)), "loop_max_us": us(max(loop)),
        "xcd_idle_frac": round(sum(max(xcd_end.values()) - v for v in xcd_end.values())
                               / (len(xcd_end) * max(xcd_end.values())), 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="w4")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--shapes", nargs="+", default=["16384,16384,1024", "16384,16384,16384"])
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--dump", default=None, help="directory for the raw traces (.pt)")
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    for shape in a.shapes:
        m, n, k = (int(v) for v in shape.split(","))
        torch.manual_seed(0)
        if dt == torch.float8_e4m3fn:
            A, _ = gemm.fp8_quantize(torch.randn(m, k, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(k, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            B = torch.randn(k, n, device="cuda", dtype=dt)
        C = torch.empty(m, n, device="cuda", dtype=gemm.out_dtype(dt))
        for kern in a.kernels.split(","):
            ms = gemm.bench_matmul(A, B, C, 10, 3, kernel=kern) / 10  # warm clocks; untraced time
            best = None
            for i in range(a.repeats):
                tr = gemm.tile_trace(A, B, kern)
                res = analyse(tr)
                if best is None or res["span_us"] < best["span_us"]:
                    best, best_tr = res, tr
            if a.dump:
                os.makedirs(a.dump, exist_ok=True)
                torch.save(best_tr, os.path.join(a.dump, f"{kern}_{m}x{n}x{k}.pt"))
            print(json.dumps({"kernel": kern, "m": m, "n": n, "k": k,
                              "untraced_us": round(ms * 1e3, 1), **best}), flush=True)
        del A, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
