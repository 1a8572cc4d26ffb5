#!/usr/bin/env python3
"""Random-shape exactness sweep of auto (every planner path: tile family,
split-K, W4 / W4S, the tail forms, the padded path): per dtype, ``--count``
shapes drawn from the sizes each dtype's fast path takes (and some it does not,
which go through the padded path or refuse), small-integer operands whose
products and sums are exact in fp32, compared with the float64 product rounded
once to the output dtype; a share of the shapes batched (2 or 3 GEMMs: the
tile order runs across the batch). One JSON line per shape; exit status 1 on
any mismatch.

    python scripts/shape_fuzz.py [--count 40] [--seed 1] [--max 7000]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402

DTYPES = ("bfloat16", "float16", "float32", "float8_e4m3fn")


def draw(rng: random.Random, dname: str, hi: int):
    """M, N, K: mostly granule multiples (the fast paths), some arbitrary."""
    g = {"float8_e4m3fn": (16, 16, 128), "float32": (4, 4, 32)}.get(dname, (8, 8, 64))
    if rng.random() < 0.25 and dname != "float8_e4m3fn":
        return rng.randint(1, hi), rng.randint(1, hi), rng.randint(1, hi)
    return tuple(rng.randint(1, max(hi // q, 1)) * q for q in g)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--count", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max", type=int, default=7000)
    ap.add_argument("--dtypes", default=",".join(DTYPES))
    ap.add_argument("--batch-frac", type=float, default=0.2, help="share of batched (bmm) shapes")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    bad = 0
    for dname in a.dtypes.split(","):
        dt = getattr(torch, dname)
        fp8 = dt == gemm.FP8
        for _ in range(a.count):
            m, n, k = draw(rng, dname, a.max)
            b = rng.choice((2, 3)) if rng.random() < a.batch_frac else 0  # 0: 2-D operands
            lead = (b,) if b else ()
            g = torch.Generator(device="cuda").manual_seed(m * 7 + n * 3 + k + b)
            lo, hi = (-2, 3) if fp8 else (-3, 4)
            Af = torch.randint(lo, hi, (*lead, m, k), device="cuda", generator=g).float()
            Bf = torch.randint(lo, hi, (*lead, k, n), device="cuda", generator=g).float()
            if fp8:
                A, B = Af.to(dt), Bf.transpose(-1, -2).contiguous().to(dt).transpose(-1, -2)
            else:
                A, B = Af.to(dt), Bf.to(dt)
            odt = gemm.out_dtype(dt)
            rec = {"dtype": dname, "m": m, "n": n, "k": k, "batch": b}
            try:
                rec["kernel"] = gemm.kernel_for(A, B)
                rec["tail"] = list(gemm.tail_split_for(A, B))
                C = gemm.matmul(A, B)
            except (RuntimeError, ValueError) as e:  # a shape no native path takes
                rec["refused"] = str(e)[:80]
                print(json.dumps(rec), flush=True)
                continue
            want = torch.matmul(Af.double(), Bf.double()).to(odt)
            d = C != want
            rec["ok"] = not bool(d.any())
            if not rec["ok"]:
                bad += 1
                idx = d.nonzero()[0].tolist()
                rec["first_bad"] = {"index": idx, "got": C[tuple(idx)].item(),
                                    "want": want[tuple(idx)].item(), "n_bad": int(d.sum().item())}
            print(json.dumps(rec), flush=True)
            del A, B, C, Af, Bf, want
    print(json.dumps({"summary": True, "bad": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
