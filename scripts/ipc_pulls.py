#!/usr/bin/env python3
"""The peer-memory collectives alone (parallel/ipc.py IpcGather), for tracing
one rank of a 2-rank gloo rehearsal on one GPU (scripts/ipc_trace2.sh): a few
all-gathers and all-reduces of 64 MiB blocks, checked, then a clean teardown.
Run with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set (one process per rank)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_matmul_benchmark_amd.parallel.comm import CommStream  # noqa: E402
from pytorch_distributed_matmul_benchmark_amd.parallel.ipc import IpcGather, ipc_empty  # noqa: E402


def main() -> int:
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    rows, cols = 4096, 8192  # 64 MiB of bf16 per rank
    src = ipc_empty((rows, cols), torch.bfloat16, dev)
    red = ipc_empty((rows, cols), torch.float32, dev)
    out = torch.empty(ws * rows, cols, dtype=torch.bfloat16, device=dev)
    g = IpcGather(CommStream(dev))
    g.register(src)
    g.register(red)
    bad = torch.zeros((), dtype=torch.int64, device=dev)  # checked on the device, read once
    for it in range(5):
        src.fill_(rank + it)
        red.fill_(float(rank + 1))
        torch.cuda.synchronize()
        g.all_gather(out, src)
        g.all_reduce(red)
        torch.cuda.synchronize()
        for r in range(ws):
            bad += (out[r * rows:(r + 1) * rows] != r + it).sum()
        bad += (red != ws * (ws + 1) / 2).sum()
    ok = int(bad.item()) == 0
    g.close()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ipc pulls {'PASS' if ok else 'FAIL'} engine {g.engine}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
