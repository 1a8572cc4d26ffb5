#!/usr/bin/env python3
"""Copy engines of the peer-memory collectives (parallel/ipc.py) on ONE GPU.

The ``--allgather ipc`` pull moves ws - 1 blocks per rank. On a node every
block comes from another GPU over its own xGMI link; on one GPU the same
calls copy device-local memory, which bounds what each engine can do (HBM,
not the link) and shows its CU cost:

  * ``kernel:B``  — ops/csrc reduce.hip ``multi_copy``: all copies in ONE
    launch, B 256-thread workgroups per copy (``PDMB_IPC_BLOCKS``; 0 = 32);
  * ``sdma:S``    — ``hipMemcpyDeviceToDeviceNoCU`` (DMA engines, no CU)
    spread over S copy streams (the sdma engine uses 2).

Each arm copies ``--copies`` blocks of ``--mib`` MiB (a 16k ws = 8 shard is 7
x 64 MiB) ``--iters`` times; interleaved rounds, median GB/s (bytes read).

    python scripts/peer_copy_bench.py [--copies 7] [--mib 64] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.ops import _native  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--copies", type=int, default=7)
    ap.add_argument("--mib", type=float, default=64.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--arms", default="kernel:8,kernel:16,kernel:32,kernel:64,sdma:1,sdma:2,sdma:7")
    a = ap.parse_args()
    mod = _native.load(build_if_missing=False)
    dev = torch.device("cuda", 0)
    n = int(a.mib * (1 << 20))
    srcs = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for _ in range(a.copies)]
    dsts = [torch.empty_like(s) for s in srcs]
    cur = torch.cuda.current_stream(dev)
    pool = [torch.cuda.Stream(device=dev) for _ in range(a.copies)]

    def run(arm: str) -> None:
        eng, _, k = arm.partition(":")
        k = int(k)
        if eng == "kernel":
            mod.peer_copy(dsts, [s.data_ptr() for s in srcs], k)
            return
        fork = torch.cuda.Event()
        fork.record(cur)
        joins = []
        for i, st in enumerate(pool[:k]):
            st.wait_event(fork)
            with torch.cuda.stream(st):
                for j in range(i, a.copies, k):
                    mod.copy_from_peer(dsts[j], srcs[j].data_ptr(), True)
            ev = torch.cuda.Event()
            ev.record(st)
            joins.append(ev)
        for ev in joins:
            cur.wait_event(ev)

    arms = a.arms.split(",")
    for arm in arms:  # warm-up, and every arm's result checked once
        for d in dsts:
            d.zero_()
        run(arm)
        torch.cuda.synchronize()
        assert all(torch.equal(s, d) for s, d in zip(srcs, dsts)), arm
    res = {arm: [] for arm in arms}
    for r in range(a.rounds):
        for arm in arms[r % len(arms):] + arms[:r % len(arms)]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(arm)
            e1.record()
            torch.cuda.synchronize()
            res[arm].append(a.copies * n * a.iters / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for arm in arms:
        eng, _, k = arm.partition(":")
        print(json.dumps({"arm": arm, "engine": eng, ("blocks_per_copy" if eng == "kernel" else "streams"): int(k),
                          "workgroups": a.copies * int(k) if eng == "kernel" else 0,
                          "copies": a.copies, "mib": a.mib, "median_gbps": round(statistics.median(res[arm]), 1),
                          "min_gbps": round(min(res[arm]), 1), "max_gbps": round(max(res[arm]), 1)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
