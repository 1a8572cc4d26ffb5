"""Direct two-shot all-reduce (parallel/comm.py ``CommStream.all_reduce_direct``)
on gloo, ws = 2 / 3 / 4: every rank must end with the same bits, equal to the
fp32 sum of the ranks' inputs in rank order rounded once to the dtype; sizes
cover empty trailing chunks (numel < ws * 64), odd lengths and 2-D row slices.
The CLI paths (batch_parallel / data_parallel / overlap with ``--allreduce
direct --check``) run end to end under torchrun."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [1, 7, 63, 130, 1000, 4099]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(rank, n, dtype):
    g = torch.Generator().manual_seed(1000 * rank + n)
    return torch.randn(n, generator=g).to(dtype)


def _worker(rank, ws, port, dtype_name, outdir):
    from pytorch_distributed_matmul_benchmark_amd.parallel.comm import CommStream

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    dtype = getattr(torch, dtype_name)
    cs = CommStream(torch.device("cpu"))
    out = {}
    for n in SIZES:
        t = _inputs(rank, n, dtype)
        cs.all_reduce_direct(t)
        out[n] = t.clone()
    # a row slice of a 2-D tensor (the overlap pipeline reduces row pieces)
    big = torch.stack([_inputs(rank, 96, dtype) for _ in range(10)])
    cs.all_reduce_direct(big[3:7])
    out["rows"] = big.clone()
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))  # files, not an mp.Queue (no socket)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3, 4, 8])
@pytest.mark.parametrize("dtype_name", ["float32", "bfloat16"])
def test_all_reduce_direct_matches_rank_order_fp32_sum(ws, dtype_name, tmp_path):
    dtype = getattr(torch, dtype_name)
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, dtype_name, str(tmp_path)))
             for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    res = {r: torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(ws)}
    for n in SIZES:
        acc = torch.zeros(n)
        for r in range(ws):
            acc += _inputs(r, n, dtype).float()
        want = acc.to(dtype)
        for r in range(ws):
            assert torch.equal(res[r][n], want), (ws, n, r)
    # rows 3..6 reduced, the others untouched
    for r in range(ws):
        mine = torch.stack([_inputs(r, 96, dtype) for _ in range(10)])
        acc = torch.zeros(4, 96)
        for q_ in range(ws):
            acc += torch.stack([_inputs(q_, 96, dtype) for _ in range(10)])[3:7].float()
        assert torch.equal(res[r]["rows"][3:7], acc.to(dtype))
        assert torch.equal(res[r]["rows"][:3], mine[:3]) and torch.equal(res[r]["rows"][7:], mine[7:])


def _torchrun(ws, script, *args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ws}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("ws,extra", [(2, []), (3, ["--overlap", "--chunks", "2"]),
                                      (4, ["--overlap", "--chunks", "1"])])
def test_batch_parallel_direct_allreduce_cli(ws, extra):
    out = _torchrun(ws, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "200",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "batch_parallel", "--allreduce", "direct", "--check", *extra)
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


def test_backup_modes_direct_allreduce_cli():
    out = _torchrun(2, "backup/matmul_distributed_benchmark.py", "--device", "cpu", "--sizes", "160",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--allreduce",
                    "direct", "--check")
    assert "PASS" in out and "FAIL" not in out
    for mode in ("no_overlap", "overlap", "pipeline"):
        out = _torchrun(2, "backup/matmul_overlap_benchmark.py", "--device", "cpu", "--sizes", "160",
                        "--iterations", "3", "--warmup", "1", "--dtype", "float32", "--mode", mode,
                        "--allreduce", "direct", "--check")
        assert "PASS" in out and "FAIL" not in out, mode


def test_bench_direct_allreduce_ws2():
    import json

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--size", "128", "--steps", "2", "--warmup", "1", "--extra-steps", "2",
                        "--extra-warmup", "1", "--allreduce", "direct"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    for key in ("batch_parallel", "batch_parallel+overlap"):
        assert d["modes"][key] and d["modes"][key]["value"] > 0, key


@pytest.mark.parametrize("extra", [[], ["--overlap", "--chunks", "2"]])
def test_matrix_parallel_ipc_allgather_cpu_falls_back_to_direct(extra):
    """--allgather ipc on CPU tensors (no peer memory) runs the direct P2P group."""
    out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "300",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "matrix_parallel", "--allgather", "ipc", "--check", *extra)
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


def test_bench_ipc_allgather_ws2_cpu():
    import json

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--size", "128", "--steps", "2", "--warmup", "1", "--extra-steps", "2",
                        "--extra-warmup", "1", "--allgather", "ipc", "--allreduce", "ipc"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    for key in ("matrix_parallel", "matrix_parallel+overlap"):
        assert d["modes"][key] and d["modes"][key]["value"] > 0, key


@pytest.mark.parametrize("extra", [[], ["--overlap", "--chunks", "2"]])
def test_batch_parallel_ipc_allreduce_cpu_falls_back_to_direct(extra):
    """--allreduce ipc on CPU tensors (no peer memory) runs the direct exchange."""
    out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "200",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "batch_parallel", "--allreduce", "ipc", "--check", *extra)
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


def test_backup_modes_ipc_allreduce_cli():
    """--allreduce ipc on the backup data_parallel and overlap family (ADVICE r3:
    data_parallel and overlap depth 1 built no comm object for ipc and raised;
    overlap depth > 1 silently ran RCCL): on CPU tensors the direct exchange
    stands in, every mode PASSes its check."""
    out = _torchrun(2, "backup/matmul_distributed_benchmark.py", "--device", "cpu", "--sizes", "160",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "data_parallel", "--allreduce", "ipc", "--check")
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
    for mode in ("no_overlap", "overlap", "pipeline"):
        out = _torchrun(2, "backup/matmul_overlap_benchmark.py", "--device", "cpu", "--sizes", "160",
                        "--iterations", "3", "--warmup", "1", "--dtype", "float32", "--mode", mode,
                        "--allreduce", "ipc", "--check")
        assert "PASS" in out and "FAIL" not in out and "ERROR" not in out, mode


def test_overlap_ipc_allreduce_uses_the_peer_path():
    """models/overlap.py with --allreduce ipc picks the peer-memory / direct
    reduce, never RCCL's (reduce_fn on the comm object make_gatherer built)."""
    import inspect

    from pytorch_distributed_matmul_benchmark_amd.models import data_parallel, overlap

    src = inspect.getsource(overlap.run)
    assert "reduce_fn(impl, comm)" in src and "cs.all_reduce_direct if" not in src
    assert "make_gatherer(impl" in inspect.getsource(data_parallel.run)


def test_auto_collective_is_measured_and_agreed():
    """--allreduce auto / --allgather auto (parallel/overlap.py pick_collective):
    every candidate that runs is timed on the job's ranks (MAX over ranks), the
    fastest is used, and the mode still checks out; bench.py reports the
    choice and the times per mode."""
    import json

    for mode, flag in (("batch_parallel", "--allreduce"), ("matrix_parallel", "--allgather")):
        for extra in ([], ["--overlap", "--chunks", "1"]):
            out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "192",
                            "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                            mode, flag, "auto", "--check", *extra)
            assert "PASS" in out and "FAIL" not in out and "ERROR" not in out, (mode, extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--size", "128", "--steps", "2", "--warmup", "1", "--extra-steps", "2",
                        "--extra-warmup", "1", "--allgather", "auto", "--allreduce", "auto"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    for key in ("batch_parallel", "batch_parallel+overlap", "matrix_parallel", "matrix_parallel+overlap"):
        m = d["modes"][key]
        assert m and m["value"] > 0, key
        c = m["collective"]
        assert c["chosen"] in ("rccl", "direct") and set(c["us"]) == {"rccl", "direct"}, (key, c)
        assert c["us"][c["chosen"]] == min(v for v in c["us"].values() if v is not None)
        assert set(c["spread_us"]) == set(c["us"])  # [min, max] over reps and ranks
        assert all(lo <= c["us"][k] <= hi for k, (lo, hi) in c["spread_us"].items())


def _pick_worker(rank, ws, port, outdir):
    import json as _json

    from pytorch_distributed_matmul_benchmark_amd.parallel import overlap as O
    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    ctx = DistContext(rank=rank, world_size=ws, local_rank=rank, device=torch.device("cpu"), backend="gloo")
    real = O.make_gatherer

    def flaky(impl, device, sources=(), comm=None):  # "direct" cannot be built on rank 1
        if impl == "direct" and rank == 1:
            raise RuntimeError("no P2P here")
        return real(impl, device, sources, comm)

    O.make_gatherer = flaky
    t = torch.full((1000,), float(rank + 1))
    impl, obj, times = O.pick_collective(ctx, "all_reduce", t, [], reps=2)
    out = torch.empty(ws * 10)
    gimpl, _, gtimes = O.pick_collective(ctx, "all_gather", torch.full((10,), float(rank)), [], reps=2)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        _json.dump({"impl": impl, "times": times, "gimpl": gimpl, "gtimes": gtimes}, f)
    dist.destroy_process_group()


def test_pick_collective_drops_a_candidate_that_fails_on_one_rank(tmp_path):
    """pick_collective: a candidate that fails on ANY rank is dropped on EVERY
    rank (times None), no rank hangs, and all ranks agree on the choice."""
    import json as _json

    ws = 3
    mp.spawn(_pick_worker, args=(ws, _port(), str(tmp_path)), nprocs=ws, join=True)
    res = [_json.load(open(tmp_path / f"r{r}.json")) for r in range(ws)]
    for r in res:
        assert r["impl"] == "rccl" and r["times"]["direct"] is None and r["times"]["rccl"] > 0
        assert r["gimpl"] == "rccl" and r["gtimes"]["direct"] is None
    assert len({_json.dumps(r, sort_keys=True) for r in res}) == 1  # identical on every rank
