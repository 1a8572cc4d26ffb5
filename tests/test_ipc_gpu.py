"""xGMI peer-memory primitives (ops/csrc/bindings.cpp ipc_*, parallel/ipc.py) on
one GPU: an ipc_empty tensor is its own allocation, its handle maps back, and a
DMA copy out of the mapping is bitwise the source. (Opening a handle in the
exporting process itself is refused by HIP, so the mapping is opened by a child
process; the 2-rank pull all-gather runs in tests/test_multirank_gpu.py.)"""
import os
import subprocess
import sys

import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import _native
from pytorch_distributed_matmul_benchmark_amd.parallel.ipc import ipc_empty

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from pytorch_distributed_matmul_benchmark_amd.ops import _native
m = _native.load(build_if_missing=False)
h = bytes.fromhex(sys.argv[2]); n = int(sys.argv[3])
addr = m.ipc_open(h, 0)
out = torch.empty(n, dtype=torch.float32, device="cuda")
m.copy_from_peer(out, addr + 4 * 16)   # from element 16 on
torch.cuda.synchronize()
m.ipc_close(addr, 0)
want = torch.arange(16, 16 + n, dtype=torch.float32, device="cuda")
print("OK" if torch.equal(out, want) else "MISMATCH")
"""


def test_ipc_empty_is_its_own_allocation_and_maps_back():
    m = _native.load(build_if_missing=False)
    t = ipc_empty((1000,), torch.float32, torch.device("cuda", 0))
    assert t.is_cuda and t.shape == (1000,) and t.is_contiguous()
    t.copy_(torch.arange(1000, dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()
    h = m.ipc_handle(t)
    assert isinstance(h, bytes) and len(h) > 0
    with pytest.raises(RuntimeError):
        m.ipc_handle(t[1:])  # not the base of its allocation
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, h.hex(), "500"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    del t
    torch.cuda.synchronize()
