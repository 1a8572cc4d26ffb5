#!/usr/bin/env python3
"""Bandwidth of the native ``reduce_sum`` kernel (ops/csrc/reduce.hip) — the local
step of the direct two-shot all-reduce (``--allreduce direct``): at ws ranks each
rank sums ws chunks of buffer/ws elements. Prints one JSON line per (dtype,
sources, chunk): median time and HBM bytes moved per second ((nsrc + 1) x chunk
bytes: every source read once, the result written once), next to a plain torch
fp32-accumulating reference of the same op (``torch.stack(...).float().sum``).

    python scripts/reduce_bench.py [--mib 64] [--srcs 2 4 8] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, nargs="+", default=[16, 64])
    ap.add_argument("--srcs", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--dtypes", nargs="+", default=["bfloat16", "float32"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    mod = _native.load(build_if_missing=False)
    for dn in a.dtypes:
        dt = getattr(torch, dn)
        for mib in a.mib:
            n = int(mib * 2 ** 20) // torch.tensor([], dtype=dt).element_size()
            for ns in a.srcs:
                srcs = [torch.randn(n, device="cuda").to(dt) for _ in range(ns)]
                out = torch.empty_like(srcs[0])
                acc = torch.zeros(n, device="cuda")
                for x in srcs:  # rank order, fp32: the kernel's semantics
                    acc += x.float()
                ref = acc.to(dt)
                del acc
                mod.reduce_sum(out, srcs)
                torch.cuda.synchronize()
                exact = bool(torch.equal(out, ref))

                def arm(native):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        if native:
                            mod.reduce_sum(out, srcs)
                        else:
                            torch.stack(srcs).float().sum(0).to(dt)
                    e1.record()
                    torch.cuda.synchronize()
                    return e0.elapsed_time(e1) / a.iters

                arm(True), arm(False)  # warm
                nat, tor = [], []
                for _ in range(a.rounds):
                    nat.append(arm(True))
                    tor.append(arm(False))
                bytes_moved = (ns + 1) * n * out.element_size()
                mn, mt = statistics.median(nat), statistics.median(tor)
                print(json.dumps({"dtype": dn, "chunk_mib": mib, "srcs": ns, "native_us": round(mn * 1e3, 1),
                                  "native_gbps": round(bytes_moved / (mn * 1e-3) / 1e9, 1),
                                  "torch_us": round(mt * 1e3, 1), "bitwise_eq_rank_order_fp32_sum": exact}),
                      flush=True)
                del srcs, out, ref
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
