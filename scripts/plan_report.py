#!/usr/bin/env python3
"""What auto runs for a shape, without a GPU (ops/csrc gemm_dispatch.cpp through
the ``plan_shape`` binding: contiguous operands at an aligned stand-in address).

For each M,N,K[,batch] and dtype, one line: the single-launch kernel and its
split-K, the model's price in microseconds, and the wave-quantisation tail form
auto takes instead, if any:

  * ``rows M1 / split S``  — rows [0, M1) unsplit, the rest split S ways;
  * ``tiles T1 / split S`` — the first T1 256x256 tiles of the tile order
    (whole waves), the rest split S ways (fp32: 128x128 tiles, f32_t128);
  * ``tiles T1 / refined xR`` — the rest cut into R smaller tiles, unsplit;
  * ``tiles T1 / stream-K (S slots)`` — fp8 stream-K (only with PDMB_STREAMK).

    python scripts/plan_report.py --dtype bfloat16 --shapes 6144,6144,6144 3072,3072,3072
    python scripts/plan_report.py --dtype float8_e4m3fn --json --shapes 4608,4608,3072
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DTYPE_IDS = {"float32": 0, "float16": 1, "bfloat16": 2, "float8_e4m3fn": 3}


def tail_form(m1: int, S: int, t1: int, r: int) -> str:
    if m1 > 0:
        return f"rows {m1} / split {S}"
    if t1 > 0 and r == 0:
        return f"tiles {t1} / stream-K ({S} slots)"
    if t1 > 0 and r > 1:
        return f"tiles {t1} / refined x{r}"
    if t1 > 0:
        return f"tiles {t1} / split {S}"
    if r == 0:  # stream-K over every tile (no whole waves first)
        return f"stream-K ({S} slots)"
    return "-"


def report(C, dtype: str, shapes, cus: int = 0):
    out = []
    for shp in shapes:
        m, n, k = shp[:3]
        b = shp[3] if len(shp) > 3 else 1
        kid, S, cost, m1, tS, t1, r = C.plan_shape(DTYPE_IDS[dtype], m, n, k, b, 0, cus)
        out.append({"dtype": dtype, "m": m, "n": n, "k": k, "batch": b, "kernel": C.kernel_name(kid),
                    "splitk": int(S), "model_us": round(float(cost), 1) if cost > 0 else None,
                    "tail": tail_form(int(m1), int(tS), int(t1), int(r))})
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dtype", default="bfloat16", choices=sorted(DTYPE_IDS))
    ap.add_argument("--shapes", nargs="+", required=True, help="M,N,K or M,N,K,batch")
    ap.add_argument("--cus", type=int, default=0, help="CU budget (0: the whole device)")
    ap.add_argument("--json", action="store_true", help="one JSON object per line")
    a = ap.parse_args(argv)
    from pytorch_distributed_matmul_benchmark_amd.ops import _native

    C = _native.load(build_if_missing=False)
    shapes = [tuple(int(v) for v in s.split(",")) for s in a.shapes]
    rows = report(C, a.dtype, shapes, a.cus)
    for r in rows:
        if a.json:
            print(json.dumps(r))
        else:
            print(f"{r['dtype']:>14} {r['m']:>6}x{r['n']}x{r['k']}"
                  f"{'x' + str(r['batch']) if r['batch'] > 1 else ''}: {r['kernel']}"
                  f" split {r['splitk']}, model {r['model_us'] if r['model_us'] else '-'} us,"
                  f" tail {r['tail']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
