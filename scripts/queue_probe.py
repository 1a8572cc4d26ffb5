#!/usr/bin/env python3
"""Hardware-queue false-dependency probe.

HIP maps a process's streams onto ``GPU_MAX_HW_QUEUES`` (4 on the pool)
hardware queues; streams that share a queue can block each other. One config
per fresh child process (queue assignment depends on the process's stream
history):

  * a gate kernel (ops gemm.SignalSet.gate: one wave polling a host flag)
    holds a "gate" stream;
  * ``waiting`` further streams wait on an event behind the gate, then each
    enqueues one op: a small kernel (``--op kernel``) or a DMA-engine copy
    (``--op sdma``: hipMemcpyDeviceToDeviceNoCU);
  * the compute (current) stream enqueues a 4096^3 bf16 GEMM;
  * ``free`` = the GEMM completed while the gate was still closed.

Prints one JSON line per config:
  {"waiting": k, "op": ..., "streams": k + 2, "free": bool, "gemm_ms": ...}
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(waiting: int, op: str, hold_s: float = 3.0) -> dict:
    import torch

    from pytorch_distributed_matmul_benchmark_amd.ops import _native, gemm

    mod = _native.load(build_if_missing=False)
    dev = torch.device("cuda", 0)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    C = torch.empty_like(A)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.empty_like(x)
    gemm.matmul(A, B, out=C)  # kernel selection / code objects loaded before the gate
    torch.cuda.synchronize()
    sig = gemm.SignalSet(dev, 1)
    gate_stream = torch.cuda.Stream(device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(waiting)]
    try:
        with torch.cuda.stream(gate_stream):
            sig.gate(0, 1, timeout_s=hold_s + 5.0)
        ev = torch.cuda.Event()
        ev.record(gate_stream)
        for st in streams:
            st.wait_event(ev)
            with torch.cuda.stream(st):
                if op == "sdma":
                    mod.copy_from_peer(y, x.data_ptr(), True)
                else:
                    y.add_(1.0)
        done = torch.cuda.Event(enable_timing=True)
        start = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        start.record()
        gemm.matmul(A, B, out=C)
        done.record()
        while not done.query() and time.perf_counter() - t0 < hold_s:
            time.sleep(0.005)
        free = bool(done.query())
        closed = not ev.query()
    finally:
        sig.set(0, 1)
        torch.cuda.synchronize()
    gemm_ms = start.elapsed_time(done)
    sig.close()
    return {"waiting": waiting, "op": op, "streams": waiting + 2, "free": free and closed,
            "gate_was_closed": closed, "gemm_ms": round(gemm_ms, 3),
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--child", nargs=2, metavar=("WAITING", "OP"))
    ap.add_argument("--waiting", type=int, nargs="+", default=[0, 1, 2, 3, 4, 6, 8])
    ap.add_argument("--ops", nargs="+", default=["kernel", "sdma"])
    a = ap.parse_args()
    if a.child:
        print(json.dumps(one(int(a.child[0]), a.child[1])), flush=True)
        return 0
    rc = 0
    for op in a.ops:
        for k in a.waiting:
            r = subprocess.run([sys.executable, __file__, "--child", str(k), op], capture_output=True,
                               text=True, timeout=120)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not line:
                print(json.dumps({"waiting": k, "op": op, "error": r.stderr[-500:]}), flush=True)
                rc = 1
                break
            print(line[-1], flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
