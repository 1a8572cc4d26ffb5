"""The overlap planner (parallel/overlap.py plan_overlap) and the pipeline's
ordering, on CPU.

Planner: on the reference's shard shapes (matmul_scaling_benchmark.py:179-188
at the default sizes :351-352) and batch units at ws = 2 / 4 / 8 it never
predicts a plan slower than serializing, refuses overlaps that cannot win
(tiny GEMMs, no collective), respects the signal granule, and honours an
explicit request. Pipeline: every GEMM it issues runs under
``gemm.shared_device()`` (or a CU budget), collectives come in unit order,
and a GEMM into a ring slot waits for that slot's previous collective."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import gemm
from pytorch_distributed_matmul_benchmark_amd.parallel import overlap as O

SIZES = (4096, 8192, 16384)


@pytest.mark.parametrize("ws", [2, 4, 8])
@pytest.mark.parametrize("n", SIZES)
def test_plan_never_predicts_worse_than_serial(ws, n):
    for kind, cols, payload in (("all_gather", n // ws, n * (n // ws) * 2),
                                ("all_reduce", n, n * n * 2)):
        for granule in (0, 16, 32):
            p = O.plan_overlap(n, cols, n, torch.bfloat16, ws, kind, payload, granule=granule)
            assert p.serial_us == pytest.approx(p.gemm_us + p.comm_us)
            if p.overlap:
                assert p.overlap_us < 0.98 * p.serial_us
                assert p.pieces in p.candidates and p.overlap_us == min(p.candidates.values())
            else:
                assert p.pieces == 1 and p.rows == 0
            tiles_m = -(-n // 256)
            if p.pieces > 1:
                assert granule > 0 and p.rows % granule == 0 and p.pieces <= tiles_m // granule
            else:
                assert p.rows == 0


def test_plan_shapes_at_16k():
    # the BASELINE config-5 shard: comm-bound at ws = 8, overlapped
    p = O.plan_overlap(16384, 2048, 16384, torch.bfloat16, 8, "all_gather", 16384 * 2048 * 2,
                       granule=32)
    assert p.overlap and p.comm_us > p.gemm_us
    # batch_parallel ws = 8: compute-bound, pieces signalled
    q = O.plan_overlap(16384, 16384, 16384, torch.bfloat16, 8, "all_reduce", 16384 ** 2 * 2,
                       granule=16)
    assert q.overlap and q.pieces > 1 and q.gemm_us > q.comm_us


def test_plan_refuses_losing_and_honours_requests():
    tiny = O.plan_overlap(256, 256, 256, torch.float32, 2, "all_reduce", 256 * 256 * 4)
    assert not tiny.overlap and "serialize" in tiny.reason
    none = O.plan_overlap(4096, 4096, 4096, torch.bfloat16, 1, "all_reduce", 4096 * 4096 * 2)
    assert not none.overlap
    forced = O.plan_overlap(256, 256, 256, torch.float32, 2, "all_reduce", 256 * 256 * 4,
                            requested=2)
    assert forced.overlap and forced.pieces == 1  # no granule: whole collectives only
    req = O.plan_overlap(16384, 16384, 16384, torch.bfloat16, 8, "all_reduce", 16384 ** 2 * 2,
                         granule=16, requested=2)
    assert req.pieces == 2 and req.rows == 32
    # measured times replace the models
    m = O.plan_overlap(16384, 2048, 16384, torch.bfloat16, 8, "all_gather", 0.0, granule=32,
                       gemm_time_us=700.0, comm_time_us=100.0)
    assert m.gemm_us == 700.0 and m.comm_us == 100.0


def test_busbw_env_override(monkeypatch):
    monkeypatch.setenv("PDMB_BUSBW_GBPS", "8:600")
    a = O.collective_us("all_reduce", 1 << 30, 8)
    monkeypatch.setenv("PDMB_BUSBW_GBPS", "8:300")
    b = O.collective_us("all_reduce", 1 << 30, 8)
    assert b > a > 0


def test_piece_rows_cover_every_row():
    for m, rows in ((16384, 16), (4352, 3), (1000, 1), (5000, 0)):
        ps = O.piece_rows(m, rows)
        assert ps[0][0] == 0 and ps[-1][1] == m
        assert all(a[1] == b[0] for a, b in zip(ps, ps[1:]))


def test_pipeline_gemms_run_shared_and_collectives_in_order():
    """Every GEMM an OverlapPipeline issues runs under gemm.shared_device (never a
    persistent kernel beside the collectives); collectives follow unit order."""
    m = 64
    A = torch.randn(m, m)
    units = [(A, A, torch.empty(m, m)) for _ in range(2)]
    seen, order = [], []

    def mm(x, y, out):
        seen.append(gemm._cus())
        torch.matmul(x, y, out=out)

    def coll(r, p, s, e, after, done):
        order.append((r, p))

    plan = O.plan_overlap(m, m, m, torch.float32, 2, "all_reduce", m * m * 4, requested=1)
    pipe = O.OverlapPipeline(mm, units, coll, torch.device("cpu"), plan, per_step=3)
    for _ in range(2):
        pipe.step()
    pipe.finish()
    assert len(seen) == 6 and all(c != 0 for c in seen)
    assert order == [(k % 2, 0) for k in range(6)]
    assert gemm._cus() == 0  # the context is left


def test_overlap_entry_points_use_the_pipeline():
    """bench.py and the models build their overlapped steps on OverlapPipeline
    (no chunked GEMM schedule remains)."""
    import inspect

    import bench
    from pytorch_distributed_matmul_benchmark_amd.models import batch_parallel, matrix_parallel

    for mod in (bench, batch_parallel, matrix_parallel):
        src = inspect.getsource(mod)
        assert "OverlapPipeline(" in src
        assert "GatherOverlap" not in src and "ReduceOverlap" not in src


def test_measured_plan_prices_the_job_from_its_own_times():
    """measured_plan (what bench.py and the modes call) times the unit's GEMM
    and one collective per candidate piece count itself: the plan carries
    those numbers (source "measured"), serial = G + C(1), and the choice
    follows them — a slow collective is overlapped, a free one serialized."""
    import time

    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    m = 64
    A = torch.randn(m, m)
    units = [(A, A, torch.empty(m, m)) for _ in range(2)]
    ctx = DistContext(rank=0, world_size=2, local_rank=0, device=torch.device("cpu"))

    def mm(x, y, out):
        time.sleep(0.004)
        torch.matmul(x, y, out=out)

    calls = []

    def slow_coll(s, e):
        calls.append((s, e))
        time.sleep(0.006)

    p = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, slow_coll, steps=10)
    assert p.source == "measured" and set(p.piece_us) == {1}
    assert 3500 < p.gemm_us < 400000 and 5000 < p.comm_us < 600000  # loose: a loaded host oversleeps
    assert p.comm_us == p.piece_us[1] and p.serial_us == pytest.approx(p.gemm_us + p.comm_us)
    assert p.overlap and calls and all(c == (0, m) for c in calls)
    free = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, lambda s, e: None, steps=10)
    assert free.source == "measured" and not free.overlap

    def broken(s, e):
        raise RuntimeError("collective unavailable")

    model = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, broken, steps=10)
    assert model.source == "model" and "measuring failed" in model.reason


def test_measured_piece_times_choose_the_piece_count():
    """With measured per-piece times the planner prices P pieces as P x one
    piece's collective: cheap pieces win, pieces with a large fixed cost lose."""
    kw = dict(granule=16, steps=10, gemm_time_us=5000.0, comm_time_us=900.0)
    cheap = O.plan_overlap(16384, 16384, 16384, torch.bfloat16, 8, "all_reduce", 0.0,
                           piece_time_us={1: 900.0, 2: 455.0, 4: 230.0}, source="measured", **kw)
    assert cheap.overlap and cheap.pieces == 4 and cheap.source == "measured"
    assert cheap.candidates[4] < cheap.candidates[2] < cheap.candidates[1]
    costly = O.plan_overlap(16384, 16384, 16384, torch.bfloat16, 8, "all_reduce", 0.0,
                            piece_time_us={1: 900.0, 2: 2000.0, 4: 1900.0}, source="measured", **kw)
    assert costly.overlap and costly.pieces == 1
    assert costly.as_dict()["piece_us"] == {"1": 900.0, "2": 2000.0, "4": 1900.0}


def test_round_comm_cus_whole_granules():
    from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import MASK_GRANULE, round_comm_cus

    assert MASK_GRANULE == 32
    assert round_comm_cus(0) == 0 and round_comm_cus(-4) == 0
    assert round_comm_cus(1) == 32 and round_comm_cus(8) == 32 and round_comm_cus(32) == 32
    assert round_comm_cus(33) == 64 and round_comm_cus(1000) == 224


def test_measured_plan_measures_the_gemm_beside_the_collective():
    """G' (VERDICT r4 #2): measured_plan times the unit's GEMM while a whole
    collective runs beside it and prices the overlap with that slowdown
    instead of the RCCL_CU_SHARE guess. Mock: a GEMM issued right behind a
    collective takes twice as long (4 -> 8 ms), so the measured share is
    (8 - 4) / min(4, 6) = 1 and the P = 1 candidate is max(G + min(G, C), C)
    + min(...) / steps."""
    import time

    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    m = 64
    A = torch.randn(m, m)
    units = [(A, A, torch.empty(m, m)) for _ in range(2)]
    ctx = DistContext(rank=0, world_size=2, local_rank=0, device=torch.device("cpu"))
    beside = [False]

    def mm(x, y, out):
        time.sleep(0.008 if beside[0] else 0.004)
        beside[0] = False

    def coll(s, e):
        time.sleep(0.006)
        beside[0] = True

    p = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, coll, steps=10, reps=5)
    assert p.source == "measured" and p.gemm_shared_us is not None
    assert p.gemm_shared_us > 1.5 * p.gemm_us
    assert 0.5 < p.cu_share <= 1.0
    G, C, s = p.gemm_us, p.comm_us, p.cu_share
    Gp = G + s * min(G, C)
    assert p.candidates[1] == pytest.approx(max(Gp, C) + min(Gp, C) / 10, rel=1e-6)
    assert p.cu_share_p == {1: p.cu_share}
    d = p.as_dict()
    assert {"gemm", "gemm_shared1", "piece1"} <= set(d["spread_us"])
    assert all(lo <= hi for lo, hi in d["spread_us"].values())
    assert d["gemm_shared_us"] == round(p.gemm_shared_us, 1)
    # the model fallback keeps the guess
    q = O.plan_overlap(16384, 2048, 16384, torch.bfloat16, 8, "all_gather", 16384 * 2048 * 2)
    assert q.gemm_shared_us is None and q.cu_share == O.RCCL_CU_SHARE


def test_plan_share_is_clamped():
    kw = dict(gemm_time_us=1000.0, comm_time_us=500.0, source="measured")
    fast = O.plan_overlap(4096, 4096, 4096, torch.bfloat16, 8, "all_reduce", 0.0,
                          gemm_shared_us=900.0, **kw)  # noise below G: no negative share
    assert fast.cu_share == 0.0
    slow = O.plan_overlap(4096, 4096, 4096, torch.bfloat16, 8, "all_reduce", 0.0,
                          gemm_shared_us=5000.0, **kw)
    assert slow.cu_share == 1.0 and not slow.overlap  # overlap can only tie serial: refused
    # per piece count: a small piece that barely disturbs the GEMM makes P = 4 win
    per = O.plan_overlap(16384, 16384, 16384, torch.bfloat16, 8, "all_reduce", 0.0, granule=16,
                         steps=10, gemm_time_us=5700.0, comm_time_us=930.0, source="measured",
                         piece_time_us={1: 930.0, 2: 283.0, 4: 152.0},
                         shared_time_us={1: 6040.0, 2: 5800.0, 4: 5720.0})
    assert per.cu_share_p[1] == pytest.approx(340 / 930) and per.cu_share_p[4] == pytest.approx(20 / 152)
    assert per.pieces == 4 and per.gemm_shared_us == 6040.0


def _fail_worker(rank, ws, port, where, outdir):
    """One rank (1) fails in measured_plan's ``where`` phase; every rank must
    return the model plan without hanging."""
    import json as _json
    import os as _os

    import torch.distributed as dist

    from pytorch_distributed_matmul_benchmark_amd.parallel import overlap as O
    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    ctx = DistContext(rank=rank, world_size=ws, local_rank=rank, device=torch.device("cpu"),
                      backend="gloo")
    m = 64
    A = torch.randn(m, m)
    units = [(A, A, torch.empty(m, m)) for _ in range(2)]
    t = torch.ones(m, m)
    calls = {"mm": 0}

    def mm(x, y, out):
        calls["mm"] += 1
        if where == "gemm" and rank == 1:
            raise RuntimeError("injected GEMM failure")
        torch.matmul(x, y, out=out)

    def prepare(s, e):  # the probe's local setup (e.g. its gather buffer): no collective
        if where == "prepare" and rank == 1:
            raise RuntimeError("injected allocation failure")

    def coll(s, e):
        dist.all_reduce(t[s:e].contiguous())

    p = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, coll, steps=10, reps=2,
                        piece_prepare=prepare)
    dist.barrier()  # every rank got here: nobody is left inside a collective
    with open(_os.path.join(outdir, f"r{rank}.json"), "w") as f:
        _json.dump({"source": p.source, "reason": p.reason}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
@pytest.mark.parametrize("where", ["gemm", "prepare"])
def test_measured_plan_one_rank_failure_is_agreed(ws, where, tmp_path):
    import json as _json
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_fail_worker, args=(ws, port, where, str(tmp_path)), nprocs=ws, join=True)
    res = [_json.load(open(tmp_path / f"r{r}.json")) for r in range(ws)]
    for r in res:
        assert r["source"] == "model" and "measuring failed" in r["reason"], r


def _plan_worker(rank, ws, port, outdir):
    """measured_plan over a real gloo group: the shared-GEMM field and the
    spread are agreed (identical on every rank)."""
    import json as _json
    import os as _os

    import torch.distributed as dist

    from pytorch_distributed_matmul_benchmark_amd.parallel import overlap as O
    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    ctx = DistContext(rank=rank, world_size=ws, local_rank=rank, device=torch.device("cpu"),
                      backend="gloo")
    m = 128
    A = torch.randn(m, m)
    units = [(A, A, torch.empty(m, m)) for _ in range(2)]
    t = torch.ones(1 << 16)

    def mm(x, y, out):
        torch.matmul(x, y, out=out)

    p = O.measured_plan(units, ctx, "all_reduce", m * m * 4, mm, lambda s, e: dist.all_reduce(t),
                        steps=10, reps=3)
    with open(_os.path.join(outdir, f"r{rank}.json"), "w") as f:
        _json.dump(p.as_dict(), f, sort_keys=True)
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
def test_measured_plan_shared_gemm_field_agreed(ws, tmp_path):
    import json as _json
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_plan_worker, args=(ws, port, str(tmp_path)), nprocs=ws, join=True)
    res = [open(tmp_path / f"r{r}.json").read() for r in range(ws)]
    assert len(set(res)) == 1  # the same plan on every rank
    d = _json.loads(res[0])
    assert d["source"] == "measured" and d["gemm_shared_us"] is not None
    assert 0.0 <= d["cu_share"] <= 1.0 and set(d["spread_us"]) == {"gemm", "gemm_shared1", "piece1"}
    G, C, s = d["gemm_us"], d["comm_us"], d["cu_share"]
    Gp = G + s * min(G, C)
    assert d["candidates"]["1"] == pytest.approx(max(Gp, C) + min(Gp, C) / 10, abs=0.2)
