#!/usr/bin/env python3
"""Interleaved A/B of native GEMM kernel variants in ONE process (cdna rule 24):
N rounds × K kernels on the same random operands; prints median/min TFLOPS per
kernel, its error vs an fp32 torch reference and whether its output is bitwise
equal to the first kernel's. The arm ``torch`` is the vendor library
(hipBLASLt: torch.matmul, or torch._scaled_mm for fp8) in the same rounds.

    python scripts/ab_kernels.py --kernels mfma256c,x_noprio --sizes 8192 16384 --rounds 5
    python scripts/ab_kernels.py --kernels auto,auto:1,torch ...    # "kernel:S": split-K S (1 = off)
    python scripts/ab_kernels.py --kernels auto,auto@PDMB_TILE_TAIL=0,torch ...  # "@VAR=VAL": env for that arm
    python scripts/ab_kernels.py --kernels fp8_w4,torch --dtype float8_e4m3fn \
        --shapes 16384,16384,2048 16384,16384,16384      # M,N,K (K sweeps: per-tile overhead)
    python scripts/ab_kernels.py --kernels auto,torch --shapes 3072,3072,3072 --sessions 3

``--sessions N`` (one session is not a result on GEMMs of tens
of microseconds, whose same-process A/B swung ~9 % between sessions): the
whole A/B runs in N fresh processes one after another; each prints its
per-kernel lines (``session``: i), then one summary line per (shape, kernel)
gives the median over sessions of the per-session medians, the min / max
session median and the ratio to the last kernel's (the vendor arm when it is
listed last) per session — the cross-session figures README / BASELINE cite.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--sizes", type=int, nargs="+", default=[8192, 16384])
    ap.add_argument("--shapes", nargs="+", default=None,
                    help="M,N,K triples or M,N,K,batch (instead of --sizes)")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--settle", type=int, default=1,
                    help="untimed runs of an arm right before each of its timed runs")
    ap.add_argument("--sessions", type=int, default=1,
                    help="repeat the whole A/B in this many fresh processes and summarise")
    a = ap.parse_args()
    if a.sessions > 1:
        return sessions(a)
    ks = a.kernels.split(",")
    dt = getattr(torch, a.dtype)
    shapes = ([tuple(int(v) for v in s.split(",")) for s in a.shapes] if a.shapes
              else [(n, n, n) for n in a.sizes])
    for shp in shapes:
        m, n, kk = shp[:3]
        bt = shp[3] if len(shp) > 3 else 0  # 0: 2-D operands
        lead = (bt,) if bt else ()
        torch.manual_seed(0)
        if dt == torch.float8_e4m3fn:  # e4m3 operands (scale 1), B column-major, bf16 C
            A, _ = gemm.fp8_quantize(torch.randn(*lead, m, kk, device="cuda"))
            B, _ = gemm.fp8_quantize(torch.randn(*lead, kk, n, device="cuda"), colmajor=True)
        else:
            A = torch.randn(*lead, m, kk, device="cuda", dtype=dt)
            B = torch.randn(*lead, kk, n, device="cuda", dtype=dt)
        C = torch.empty(*lead, m, n, device="cuda", dtype=gemm.out_dtype(dt))
        flops = 2.0 * m * n * kk * max(bt, 1)
        one = torch.ones((), device="cuda")

        def vendor(out=None):
            if dt == torch.float8_e4m3fn:
                return torch._scaled_mm(A, B, one, one, out_dtype=torch.bfloat16, out=out)
            return torch.matmul(A, B, out=out)

        def arm(k):  # "kernel", "kernel:S" (S = K slices: split-K forced / off with 1),
            # either with "@VAR=VAL" (an environment switch the dispatcher reads per call)
            k, _, env = k.partition("@")
            name, _, S = k.partition(":")
            return name, int(S or 0), env

        class envset:  # the arm's environment switch for the duration of its calls
            def __init__(self, env):
                self.kv = env.split("=", 1) if env else None

            def __enter__(self):
                if self.kv:
                    self.old = os.environ.get(self.kv[0])
                    os.environ[self.kv[0]] = self.kv[1]

            def __exit__(self, *exc):
                if self.kv:
                    if self.old is None:
                        os.environ.pop(self.kv[0], None)
                    else:
                        os.environ[self.kv[0]] = self.old

        def run(k):
            if k == "torch":
                return vendor()
            name, S, env = arm(k)
            with envset(env):
                return gemm.matmul(A, B, kernel=name, splitk=S)

        def bench(k, iters):
            if k != "torch":
                name, S, env = arm(k)
                with envset(env):
                    return gemm.bench_matmul(A, B, C, iters, 2, kernel=name, splitk=S) / iters
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            vendor(C)
            e0.record()
            for _ in range(iters):
                vendor(C)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / iters

        ref = run(ks[0])
        R = torch.matmul(A.float(), B.float())
        errs, same = {}, {}
        shape_ks = []
        for k in ks:
            try:
                out = run(k)
            except RuntimeError as e:  # e.g. a forced split this K cannot take
                print(json.dumps({"n": n, **({"m": m, "k": kk} if a.shapes else {}), "kernel": k,
                                  "skipped": str(e)}), flush=True)
                continue
            shape_ks.append(k)
            errs[k] = ((out.float() - R).norm() / R.norm()).item()  # diag_* builds are timing-only
            same[k] = bool(torch.equal(out, ref))
        for _ in range(2):  # warm clocks
            for k in shape_ks:
                bench(k, 5)
        res = {k: [] for k in shape_ks}
        for r in range(a.rounds):
            # rotate the arm order every round: no arm always runs first (right
            # after the previous round's last arm), which biased the medians by
            # a few % on short kernels (profiles/r3_ldc_probe_*.jsonl)
            for k in shape_ks[r % len(shape_ks):] + shape_ks[:r % len(shape_ks)]:
                # untimed runs of the same arm first: rotation keeps the cyclic
                # order, so without them an arm always times right after the same
                # predecessor (the arm after hipBLASLt measured up to 3 % low on
                # fp32 with an identical plan, profiles/r7af_*)
                for _ in range(a.settle):
                    bench(k, a.iters)
                res[k].append(flops / bench(k, a.iters) / 1e9)
        for k in shape_ks:
            med = statistics.median(res[k])
            print(json.dumps({"n": n, **({"m": m, "k": kk} if a.shapes else {}),
                              **({"batch": bt} if bt else {}), "kernel": k,
                              "median_tflops": round(med, 1), "median_us": round(flops / med / 1e6, 1),
                              "min": round(min(res[k]), 1), "max": round(max(res[k]), 1),
                              "relerr": errs[k], "bitwise_eq_first": same[k]}), flush=True)
        del A, B, C, ref, R
        torch.cuda.empty_cache()


def sessions(a) -> int:
    """Run the A/B in ``a.sessions`` fresh child processes and summarise."""
    import subprocess

    argv = [x for x in sys.argv[1:]]
    i = argv.index("--sessions")
    del argv[i:i + 2]
    runs = []
    for sid in range(a.sessions):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), *argv], capture_output=True,
                           text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr[-3000:])
            return r.returncode
        recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        for d in recs:
            d["session"] = sid
            print(json.dumps(d), flush=True)
        runs.append([d for d in recs if "median_tflops" in d])  # not the skipped arms
    kernels = a.kernels.split(",")
    last = kernels[-1]
    keys = [(d.get("m"), d["n"], d.get("k"), d.get("batch"), d["kernel"]) for d in runs[0]]
    for key in keys:
        meds, ratios = [], []
        for recs in runs:
            by = {(d.get("m"), d["n"], d.get("k"), d.get("batch"), d["kernel"]): d for d in recs}
            meds.append(by[key]["median_tflops"])
            ref = by.get(key[:4] + (last,))
            if ref:
                ratios.append(by[key]["median_tflops"] / ref["median_tflops"])
        m, n, k, b, kern = key
        print(json.dumps({"summary": True, "n": n, **({"m": m, "k": k} if m is not None else {}),
                          **({"batch": b} if b else {}), "kernel": kern, "sessions": len(meds),
                          "session_medians": meds, "median_tflops": round(statistics.median(meds), 1),
                          "min_session": min(meds), "max_session": max(meds),
                          "ratio_vs": last, "ratio_per_session": [round(x, 4) for x in ratios],
                          "ratio_median": round(statistics.median(ratios), 4) if ratios else None}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
