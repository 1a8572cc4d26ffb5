#!/usr/bin/env python3
"""The overlap schedule against serialization, measured on ONE GPU with a comm proxy.

A collective's cost on the GPU that runs it is (a) time on its own stream and
(b) CUs and HBM taken from the GEMM beside it. RCCL cannot run with one rank,
so the proxy (ops.gemm.comm_proxy: a 16-B copy with a fixed number of
256-thread workgroups, like an RCCL collective's channels, HBM-bound like its
copy loop) stands in for the collective of every unit; everything else is the
production schedule: parallel/overlap.py OverlapPipeline with its ring of
outputs and, for pieces > 1, the W4 kernel's completion signals.

Units (one GEMM each, VERDICT r2 "Next round" #1):
  shard  [16384 x 16384] @ [16384 x 2048]   matrix_parallel's ws = 8 shard
  batch  [16384 x 16384] @ [16384 x 16384]  batch_parallel's ws = 8 unit
Proxy bytes per unit: --proxy-mib (default 16 and 256): a compute-bound and a
comm-bound step.

Arms (interleaved rounds, best of each; ms per unit over --units units):
  gemm       the unit's GEMM alone, best kernel (auto on a quiet device)
  proxy      the proxy alone on the high-priority comm stream
  serial     GEMM then proxy, on one stream (unchunked serialization)
  pipe_P     OverlapPipeline with P pieces (P = 1: whole-unit proxies
             pipelined across units; P > 1: signalled pieces)
Reported: speedup = serial / arm, the GEMM rate the schedule sustains
(unit FLOPs / arm time, meaningful where the step is compute-bound), and
the planner's choice with its distance from the best measured arm. The
planner is the production one, ``measured_plan`` (parallel/overlap.py): it
times the unit's GEMM and one proxy piece per candidate piece count itself,
exactly as the modes do on their ranks (``plan`` in the record, source
"measured"); ``plan_model`` is the table-model plan for comparison.

    python scripts/overlap_proxy.py [--units 10] [--rounds 3] [--proxy-mib 16 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import gemm  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.comm import CommStream  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import (  # noqa: E402
    OverlapPipeline, compute_ctx, compute_stream, measured_plan, plan_overlap)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--shapes", nargs="+", default=["shard", "batch"])
    ap.add_argument("--proxy-mib", type=float, nargs="+", default=[16.0, 256.0])
    ap.add_argument("--proxy-blocks", type=int, default=32)
    ap.add_argument("--pieces", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--units", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--comm-cus", type=int, nargs="+", default=[0],
                    help="also run every pipe_P with the GEMMs on a stream whose CU mask leaves "
                         "k CUs to the proxy (arms pipe_P_cuK, gemm_cuK; 0 = no mask)")
    ap.add_argument("--piece-us", type=float, default=10.0,
                    help="planner: cost of one more piece (host flag wait + proxy launch)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    n = a.n
    cstream = CommStream(dev)  # high priority, as the modes' comm stream
    comm = cstream.stream
    # the planner's view of the job: 8 ranks (no process group: its MAX over
    # ranks is this process's own measurement)
    ctx8 = DistContext(rank=0, world_size=8, local_rank=0, device=dev)
    cur = torch.cuda.current_stream(dev)

    def rnd(*shape, seed):
        g.manual_seed(seed)
        return torch.randn(*shape, generator=g, device=dev, dtype=torch.bfloat16)

    def timed(fn, units):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(units)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / units

    for shape in a.shapes:
        ncols = n // 8 if shape == "shard" else n
        A = rnd(n, n, seed=1)
        B = rnd(n, ncols, seed=2)
        Cs = [torch.empty(n, ncols, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        units = [(A, B, Cs[0]), (A, B, Cs[1])]
        flops = 2.0 * n * n * ncols
        with gemm.shared_device():
            granule = gemm.signal_granule(A, B, Cs[0])
            shared_kernel = gemm.kernel_for(A, B, Cs[0])
        alone_kernel = gemm.kernel_for(A, B, Cs[0])
        for mib in a.proxy_mib:
            el = int(mib * (1 << 20) / 2) // 8 * 8
            src = torch.randn(el, device=dev, dtype=torch.bfloat16)
            dst = torch.empty_like(src)

            def proxy(s, e):  # the rows [s, e) of a unit's output: that share of the bytes
                lo, hi = (el * s // n) // 8 * 8, (el * e // n) // 8 * 8
                if hi > lo:
                    gemm.comm_proxy(dst[lo:hi], src[lo:hi], a.proxy_blocks)

            def coll(r, p, s, e, after, done):
                with torch.cuda.stream(comm):
                    if after is not None:
                        comm.wait_event(after)
                    proxy(s, e)
                    if done is not None:
                        done.record(comm)

            def run_gemm(k):
                for i in range(k):
                    gemm.matmul(A, B, out=Cs[i % 2])

            def run_proxy(k):
                comm.wait_stream(cur)
                with torch.cuda.stream(comm):
                    for _ in range(k):
                        proxy(0, n)
                cur.wait_stream(comm)

            def run_serial(k):
                for i in range(k):
                    gemm.matmul(A, B, out=Cs[i % 2])
                    proxy(0, n)

            pipes = {}
            for P in a.pieces:
                plan = plan_overlap(n, ncols, n, torch.bfloat16, 8, "all_gather", 0.0,
                                    granule=granule, requested=P, gemm_time_us=1.0,
                                    comm_time_us=1.0)
                plan.overlap = True
                if P > 1 and plan.pieces != P:
                    continue  # the granule does not allow P pieces
                pipes[P] = OverlapPipeline(lambda x, y, o: gemm.matmul(x, y, out=o), units, coll,
                                           dev, plan, per_step=1, compute=cur, comm=None)

            def run_pipe(pipe, stream=None):
                def f(k):
                    if stream is not None:
                        stream.wait_stream(cur)
                    for _ in range(k):
                        pipe.step()
                    pipe.finish()
                    if stream is not None:
                        cur.wait_stream(stream)
                return f

            arms = {"gemm": run_gemm, "proxy": run_proxy, "serial": run_serial}
            for P in pipes:
                arms[f"pipe_{P}"] = run_pipe(pipes[P])
            owners = []
            for cus in (c for c in a.comm_cus if c > 0):
                stream, owner = compute_stream(dev, cus)
                owners.append(owner)

                def run_gemm_masked(k, stream=stream, owner=owner):
                    stream.wait_stream(cur)
                    with compute_ctx(stream, owner):
                        for i in range(k):
                            gemm.matmul(A, B, out=Cs[i % 2])
                    cur.wait_stream(stream)
                arms[f"gemm_cu{cus}"] = run_gemm_masked
                for P in [q for q in pipes if isinstance(q, int)]:
                    pm = OverlapPipeline(lambda x, y, o: gemm.matmul(x, y, out=o), units, coll, dev,
                                         pipes[P].plan, per_step=1, compute=stream, owner=owner,
                                         comm=None)
                    pipes[(P, cus)] = pm
                    arms[f"pipe_{P}_cu{cus}"] = run_pipe(pm, stream)
            for f in arms.values():  # warm-up: clocks, allocator, counters, signals
                f(2)
            best = {}
            for _ in range(a.rounds):
                for name, f in arms.items():
                    best[name] = min(best.get(name, 1e9), timed(f, a.units))
            G, Cp, S = best["gemm"], best["proxy"], best["serial"]

            def probe(s, e):
                with torch.cuda.stream(comm):
                    proxy(s, e)
            plan = measured_plan(units, ctx8, "all_gather", 0.0,
                                 lambda x, y, o: gemm.matmul(x, y, out=o), probe, steps=a.units,
                                 compute=cur, comm=cstream, reps=5)
            model = plan_overlap(n, ncols, n, torch.bfloat16, 8, "all_gather", 0.0, granule=granule,
                                 steps=a.units, gemm_time_us=G * 1e3, comm_time_us=Cp * 1e3,
                                 piece_us=a.piece_us)
            arm_best = min((k for k in best if k.startswith("pipe_") and "_cu" not in k),
                           key=lambda k: best[k])
            chosen = f"pipe_{plan.pieces}" if plan.overlap else "serial"
            rec = {"shape": shape, "m": n, "n": ncols, "k": n, "proxy_mib": mib,
                   "proxy_blocks": a.proxy_blocks, "units": a.units, "granule": granule,
                   "kernel_alone": alone_kernel, "kernel_shared": shared_kernel,
                   "ms": {k: round(v, 4) for k, v in best.items()},
                   "gemm_tflops_alone": round(flops / G / 1e9, 1),
                   "speedup_vs_serial": {k: round(S / v, 3) for k, v in best.items()
                                         if k.startswith("pipe_")},
                   "tflops_in_schedule": {k: round(flops / v / 1e9, 1) for k, v in best.items()
                                          if k.startswith("pipe_")},
                   "best_arm": arm_best, "planner": chosen, "plan": plan.as_dict(),
                   # the GEMM's measured slowdown beside one whole proxy collective
                   "gemm_shared_over_gemm": (round(plan.gemm_shared_us / plan.gemm_us, 4)
                                             if plan.gemm_shared_us else None),
                   "plan_model": model.as_dict(),
                   "planner_vs_best": round(best.get(chosen, S) / best[arm_best], 4)}
            print(json.dumps(rec), flush=True)
            for p in pipes.values():
                p.close()
            for o in owners:
                o.close()
            del src, dst
        del A, B, Cs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
