"""xGMI peer-memory primitives (ops/csrc/bindings.cpp ipc_* / peer_copy /
reduce_sum_addrs, parallel/ipc.py) on one GPU: an ipc_empty tensor is its own
allocation, its handle maps back, and a DMA copy out of the mapping is bitwise
the source; the one-launch multi-peer copy and the by-address sum are bitwise;
a rank's stream set has no false hardware-queue dependency. (Opening a handle
in the exporting process itself is refused by HIP, so the mapping is opened by
a child process; the multi-rank pulls run in tests/test_multirank_gpu.py.)"""
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


DEV = torch.device("cuda", 0)


def test_peer_copy_one_launch_bitwise():
    """reduce.hip multi_copy: several copies (odd lengths, an unaligned source,
    an empty one) in one launch are bitwise the sources, for default and
    explicit workgroup counts."""
    m = _native.load(build_if_missing=False)
    g = torch.Generator(device="cuda").manual_seed(7)
    lens = [1, 15, 16, 4097, 1 << 20, (3 << 20) + 5, 0]
    srcs = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=DEV, generator=g) for n in lens]
    big = torch.randint(0, 256, (1 << 16,), dtype=torch.uint8, device=DEV, generator=g)
    srcs.append(big[3:])  # a 16-B-unaligned source: the byte path
    for blocks in (0, 1, 5):
        dsts = [torch.full((s.numel(),), 0xAB, dtype=torch.uint8, device=DEV) for s in srcs]
        m.peer_copy(dsts, [s.data_ptr() for s in srcs], blocks)
        torch.cuda.synchronize()
        for s, d in zip(srcs, dsts):
            assert torch.equal(s, d), (blocks, s.numel())
    with pytest.raises(RuntimeError):
        m.peer_copy([torch.empty(4, device=DEV)] * (m.MAX_COPIES + 1), [1] * (m.MAX_COPIES + 1), 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_reduce_sum_addrs_matches_reduce_sum(dtype):
    """The fused pull + sum of the peer-memory all-reduce (sources by address)
    is bitwise the tensor-list reduce_sum, with and without a grid cap."""
    m = _native.load(build_if_missing=False)
    g = torch.Generator(device="cuda").manual_seed(11)
    srcs = [torch.randn(1_000_003, device=DEV, dtype=dtype, generator=g) for _ in range(8)]
    ref = torch.empty_like(srcs[0])
    m.reduce_sum(ref, srcs)
    for blocks in (0, 3):
        out = torch.empty_like(ref)
        m.reduce_sum_addrs(out, [s.data_ptr() for s in srcs], blocks)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), blocks
    want = torch.stack([s.float() for s in srcs]).sum(0)
    assert torch.allclose(ref.float(), want, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("sdma", [True, False])
def test_copy_from_peer_kinds_bitwise(sdma):
    """copy_from_peer: the NoCU (DMA engine) kind and the plain kind copy the same bytes."""
    m = _native.load(build_if_missing=False)
    src = torch.randn(3 << 20, device=DEV)
    dst = torch.zeros_like(src)
    m.copy_from_peer(dst, src.data_ptr(), sdma)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)


def test_gate_holds_the_stream_until_released():
    """ops gemm.SignalSet.gate: the stream stays blocked until the host sets the flag."""
    import time

    from pytorch_distributed_matmul_benchmark_amd.ops import gemm

    sig = gemm.SignalSet(DEV, 1)
    st = torch.cuda.Stream(device=DEV)
    try:
        with torch.cuda.stream(st):
            sig.gate(0, 1, timeout_s=20.0)
        ev = torch.cuda.Event()
        ev.record(st)
        time.sleep(0.3)
        held = not ev.query()
    finally:
        sig.set(0, 1)
    t0 = time.perf_counter()
    ev.synchronize()
    assert held and time.perf_counter() - t0 < 10.0
    sig.close()


def test_rank_stream_set_has_no_false_queue_dependency():
    """A rank's streams under --allgather/--allreduce ipc (kernel engine): the
    compute stream, the comm stream and ProcessGroupNCCL's internal stream —
    modelled as a gate stream plus two streams waiting behind it — fit the
    process's 4 hardware queues: a GEMM on the compute stream completes while
    the others are blocked (scripts/queue_probe.py, one fresh process; the
    gate releases itself after a timeout, so this cannot hang)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "queue_probe.py"), "--child", "2",
                        "kernel"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = __import__("json").loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["gate_was_closed"] and d["free"], d


def test_ipc_handle_reuse_and_the_pool():
    """scripts/ipc_handle_probe.py (two processes): with hipFree between
    exports (PDMB_IPC_ARENA=0) a buffer re-allocated at the freed address is
    exported under the same handle bytes, and — what made the pre-arena churn
    unsafe — a peer still holding the old import gets that stale mapping back
    (recorded, profiles/r7c_ipc_handle_probe.jsonl). The pool (default) hands
    the same live buffer back under the same handle while the peer keeps its
    mapping: every read current."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ipc_handle_probe.py"),
                        "--trials", "3"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [__import__("json").loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    trials = [x for x in recs if "trial" in x]
    bypass = [x for x in trials if not x["arena"]]
    pool = [x for x in trials if x["arena"]]
    # equal-size churn, child closing first: handles repeat with the address, reads are current
    same_size = [x for x in bypass[1:3]]
    assert all(x["same_handle_as_prev"] == x["same_ptr_as_prev"] for x in same_size), same_size
    assert all(x.get("read_ok") for x in bypass[:3]), bypass[:3]
    # the pool: same buffer, same handle, the peer's open mapping reads the new bytes
    assert len(pool) == 3 and all(x.get("read_ok") for x in pool), pool
    assert all(x["same_ptr_as_prev"] and x["same_handle_as_prev"] for x in pool[1:]), pool
