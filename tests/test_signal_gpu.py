"""W4 completion signals (gemm_w4.hip SIG, common.h signal_tile) and the overlap
pipeline built on them (parallel/overlap.py OverlapPipeline).

* a signalled launch writes the same C as the plain one, bit for bit (the
  write-through epilogue stores the same bf16 words);
* every slot's host flag reaches the launch's epoch, and the device counters
  keep counting across launches (launch e completes a slot at e x tiles);
* hand-off under load: a consumer stream copies each piece the moment its
  flag arrives while the same launch still computes, from a consumer whose
  caches hold the buffer's previous contents; every copied word must equal
  the finished C (a stale read shows up as a mismatch);
* the pipeline with a proxy collective: ring slots, WAR waits and signalled
  pieces leave every output equal to the plain GEMM."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import gemm
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import (OverlapPipeline, piece_rows,
                                                                        plan_overlap)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ints(*shape, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(-3, 4, shape, device="cuda", generator=g).to(torch.bfloat16)


def _rnd(*shape, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(*shape, device="cuda", generator=g, dtype=torch.bfloat16)


@pytest.mark.parametrize("m,n,k,rows,splitk", [
    (4096, 4096, 2048, 4, 0),   # 256 tiles, supertile order
    (8192, 1024, 4096, 8, 0),   # thin grid (matrix_parallel shard shape)
    (4096, 4096, 4096, 2, 2),   # split-K: only the slice that writes C signals
    (4352, 2560, 1024, 3, 1),   # edge tiles in M and N, last slot short
])
def test_signalled_gemm_matches_and_flags(m, n, k, rows, splitk):
    A, B = _rnd(m, k, seed=1), _rnd(k, n, seed=2)
    ref = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    kw = {"kernel": "w4", "splitk": splitk}
    with gemm.shared_device():
        gemm.matmul(A, B, out=ref, **kw)
        assert gemm.signal_granule(A, B, ref, kernel="w4") > 0
    tm = -(-m // 256)
    slots = -(-tm // rows)
    sig = gemm.SignalSet(DEV, slots)
    try:
        out = torch.full((m, n), float("nan"), device=DEV, dtype=torch.bfloat16)
        for e in (1, 2, 3):
            out.fill_(float("nan"))
            with gemm.shared_device():
                gemm.matmul(A, B, out=out, signal=(sig, rows, sig.next_epoch()), **kw)
            for s in range(slots):
                sig.wait(s, e, timeout_s=30.0)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), f"launch {e}"
            assert all(sig.flag(s) == e for s in range(slots))
    finally:
        sig.close()


def test_signal_refuses_non_w4():
    A, B = _rnd(512, 512, seed=3), _rnd(512, 512, seed=4)
    out = torch.empty(512, 512, device=DEV, dtype=torch.bfloat16)
    sig = gemm.SignalSet(DEV, 4)
    try:
        with pytest.raises(RuntimeError):
            gemm.matmul(A, B, out=out, kernel="t128", signal=(sig, 1, sig.next_epoch()))
    finally:
        sig.close()
    assert gemm.signal_granule(A.float(), B.float()) == 0


def test_handoff_consumer_sees_finished_pieces_under_load():
    """Pieces copied by a consumer stream as their flags arrive (while the launch
    still runs, with a second GEMM loading the chip) equal the final C."""
    m, n, k, rows = 8192, 4096, 4096, 8
    A, B = _ints(m, k, seed=5), _ints(k, n, seed=6)
    A2, B2 = _rnd(4096, 4096, seed=7), _rnd(4096, 4096, seed=8)
    C2 = torch.empty(4096, 4096, device=DEV, dtype=torch.bfloat16)
    out = torch.zeros(m, n, device=DEV, dtype=torch.bfloat16)
    snap = torch.empty_like(out)
    pieces = piece_rows(m, rows)
    sig = gemm.SignalSet(DEV, len(pieces))
    consumer = torch.cuda.Stream(device=DEV)
    load = torch.cuda.Stream(device=DEV)
    try:
        for trial in range(3):
            out.fill_(trial + 7)  # stale contents the consumer reads first (caches warm)
            consumer.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(consumer):
                snap.copy_(out)
            torch.cuda.synchronize()
            epoch = sig.next_epoch()
            with gemm.shared_device():
                gemm.matmul(A, B, out=out, signal=(sig, rows, epoch))
                with torch.cuda.stream(load):
                    gemm.matmul(A2, B2, out=C2)
            early = 0
            for p, (s, e) in enumerate(pieces):
                sig.wait(p, epoch, timeout_s=30.0)
                early += int(not torch.cuda.current_stream().query())
                with torch.cuda.stream(consumer):
                    snap[s:e].copy_(out[s:e])
            torch.cuda.synchronize()
            assert torch.equal(snap, out), f"trial {trial}: a piece was read stale"
        R = (A.double() @ B.double()).to(torch.bfloat16)
        assert torch.equal(out, R)
        assert early >= 1  # at least one piece was handed off while the GEMM still ran
    finally:
        sig.close()


def _proxy_pipeline(pieces, steps=5):
    """OverlapPipeline over a 2-slot ring with a copy kernel as the 'collective'
    and a distinct A per unit (the operands hook): returns, per ring slot, the
    unit that last wrote it, its GEMM output, its copy and that unit's product."""
    m, n, k = 8192, 4096, 2048
    As = [_ints(m, k, seed=100 + i) for i in range(steps)]
    B = _ints(k, n, seed=10)
    units = [(As[0], B, torch.empty(m, n, device=DEV, dtype=torch.bfloat16)) for _ in range(2)]
    copies = [torch.zeros(m, n, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    comm = torch.cuda.Stream(device=DEV, priority=-1)
    with gemm.shared_device():
        granule = gemm.signal_granule(As[0], B, units[0][2])
    plan = plan_overlap(m, n, k, torch.bfloat16, 8, "all_gather", 0.0, granule=granule,
                        requested=pieces, gemm_time_us=1.0, comm_time_us=1.0)
    issued = []

    def coll(r, p, s, e, after, done):
        with torch.cuda.stream(comm):
            if after is not None:
                comm.wait_event(after)
            copies[r][s:e].copy_(units[r][2][s:e])
            if done is not None:
                done.record(comm)
        issued.append((r, p, s, e))

    pipe = OverlapPipeline(lambda x, y, o: gemm.matmul(x, y, out=o), units, coll, DEV, plan,
                           per_step=1, compute=torch.cuda.current_stream(DEV),
                           operands=lambda i: (As[i], B))
    try:
        assert pipe.signalled == (pieces > 1 and plan.pieces > 1)
        for _ in range(steps):
            pipe.step()
        pipe.finish()
        torch.cuda.synchronize()
        assert len(issued) == steps * len(pipe.pieces)
        out = []
        for r in range(2):
            u = pipe.slot_unit[r]
            R = (As[u].double() @ B.double()).to(torch.bfloat16)
            out.append((u, units[r][2], copies[r], R))
        return out, pipe.signalled
    finally:
        pipe.close()


@pytest.mark.parametrize("pieces", [1, 2, 4])
def test_pipeline_with_proxy_collective(pieces):
    """Every unit has its own product; after the run each ring slot holds the
    last unit that wrote it (units 3 and 4 of 5), and the 'collective' copied
    exactly that unit's finished GEMM — whole and signalled pieces."""
    slots, _ = _proxy_pipeline(pieces)
    assert sorted(u for u, *_ in slots) == [3, 4]
    for u, out, copy, R in slots:
        assert torch.equal(out, R), u
        assert torch.equal(copy, R), u


@pytest.mark.parametrize("pieces", [1, 2])
def test_pipeline_negative_control_catches_a_skipped_wait(pieces, monkeypatch):
    """Negative control for the check above: with the producer dependency
    removed (PDMB_TEST_SKIP_READY_WAIT: no ready event, no signal wait, each
    GEMM delayed on the compute stream) the copies read the slots' previous
    units, and the same comparison fails."""
    monkeypatch.setenv("PDMB_TEST_SKIP_READY_WAIT", "20000000")
    slots, _ = _proxy_pipeline(pieces)
    assert any(not torch.equal(copy, R) for u, out, copy, R in slots)
    for u, out, copy, R in slots:
        assert torch.equal(out, R), u  # the GEMMs themselves are still right
