"""Multi-rank GPU code paths on a single-GPU box: two torchrun ranks share the
GPU over the gloo backend (RCCL refuses two ranks on one device), so the
CommStream event ordering, overlap chunking, padded shards and the float64
Σ-over-ranks checks run with real HIP streams and the native kernels."""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(nproc, script, *args, port=None, env=None):
    port = port or free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1", **(env or {}))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
                        f"--master-port={port}", script, "--dist-backend", "gloo", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _records(path):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


@pytest.mark.parametrize("mode,extra", [("batch_parallel", []), ("batch_parallel", ["--overlap"]),
                                        ("matrix_parallel", []),
                                        ("matrix_parallel", ["--overlap", "--chunks", "2"]),
                                        ("ring_parallel", [])])
def test_two_ranks_share_gpu_scaling_modes(mode, extra):
    out = _run(2, "matmul_scaling_benchmark.py", "--sizes", "2048", "4608", "--iterations", "3",
               "--warmup", "1", "--mode", mode, "--check", *extra)
    assert "Collective operations verified successfully across 2 GPUs" in out
    assert out.count("PASS") == 2 and "FAIL" not in out and "ERROR" not in out


@pytest.mark.parametrize("mode", ["data_parallel", "model_parallel"])
def test_two_ranks_share_gpu_backup_distributed(mode):
    out = _run(2, "backup/matmul_distributed_benchmark.py", "--sizes", "2048", "--iterations", "2",
               "--warmup", "1", "--mode", mode, "--check")
    assert "PASS" in out and "ERROR" not in out


@pytest.mark.parametrize("mode", ["overlap", "pipeline"])
def test_two_ranks_share_gpu_overlap_ring(mode):
    out = _run(2, "backup/matmul_overlap_benchmark.py", "--sizes", "2048", "--iterations", "4",
               "--warmup", "1", "--mode", mode, "--check")
    assert "PASS" in out and "ERROR" not in out


def test_two_ranks_share_gpu_bench_json():
    out = _run(2, "bench.py", "--gpus", "2", "--size", "2048", "--steps", "3", "--warmup", "1",
               "--mode", "batch_parallel", "--overlap")
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0
    # the secondary modes ran on the same ranks: the other three scaling variants
    assert set(d["modes"]) == {"batch_parallel", "matrix_parallel", "matrix_parallel+overlap"}
    assert all(m["value"] > 0 for m in d["modes"].values())


def test_two_ranks_share_gpu_bench_ring():
    out = _run(2, "bench.py", "--gpus", "2", "--size", "2048", "--steps", "3", "--warmup", "1",
               "--mode", "ring_parallel", "--extra-steps", "0")
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "ring2"


@pytest.mark.parametrize("mode,extra", [
    ("matrix_parallel", ["--overlap", "--chunks", "4", "--comm-cus", "16"]),
    ("batch_parallel", ["--overlap", "--chunks", "2", "--comm-cus", "32"]),
    ("matrix_parallel", ["--overlap", "--chunks", "1"]),
    ("batch_parallel", ["--overlap", "--chunks", "4", "--batch", "2"]),
    ("matrix_parallel", ["--allgather", "direct"]),
    ("matrix_parallel", ["--allgather", "direct", "--overlap", "--chunks", "2"]),
    ("matrix_parallel", ["--allgather", "ipc"]),
    ("matrix_parallel", ["--allgather", "ipc", "--overlap", "--chunks", "1"]),
    ("matrix_parallel", ["--allgather", "ipc", "--overlap", "--chunks", "2"]),
    ("batch_parallel", ["--allreduce", "ipc"]),
    ("batch_parallel", ["--allreduce", "ipc", "--overlap", "--chunks", "1"]),
    ("batch_parallel", ["--allreduce", "ipc", "--overlap", "--chunks", "2", "--batch", "2"]),
    ("batch_parallel", ["--allreduce", "direct"]),
    ("batch_parallel", ["--allreduce", "direct", "--overlap", "--chunks", "2"])])
def test_two_ranks_cu_masked_overlap_checked(mode, extra):
    """The overlap pipeline (ring of outputs; signalled pieces where --chunks > 1
    and the GEMM is W4), optionally on a CU-masked stream: the float64
    Σ-over-ranks / gathered-C checks still pass."""
    out = _run(2, "matmul_scaling_benchmark.py", "--sizes", "2048", "--iterations", "3",
               "--warmup", "1", "--mode", mode, "--check", *extra)
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


def test_two_ranks_self_launch_through_bench():
    """bench.py --gpus 2 with no torchrun starts both ranks itself (gloo: they share
    the one GPU) and reports a scaling efficiency against rank 0 alone."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo",
                        "--size", "2048", "--steps", "3", "--warmup", "1", "--extra-steps", "2",
                        "--extra-warmup", "1", "--comm-cus", "16"], cwd=ROOT, capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["single_gpu_tflops"] > 0
    assert d["scaling_efficiency"] is not None
    assert d["modes"]["matrix_parallel+overlap"]["value"] > 0


def test_two_ranks_share_gpu_bench_ipc_allgather():
    """bench.py with --allgather ipc at ws = 2 (both ranks on one GPU, gloo): the
    peer-memory pull runs in matrix_parallel serialized and overlapped and the
    IpcGather teardown (unmap + barrier) leaves the job exiting cleanly."""
    out = _run(2, "bench.py", "--gpus", "2", "--size", "2048", "--steps", "3", "--warmup", "1",
               "--extra-steps", "2", "--extra-warmup", "1", "--allgather", "ipc", "--allreduce", "ipc")
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    for key in ("matrix_parallel", "matrix_parallel+overlap", "batch_parallel", "batch_parallel+overlap"):
        assert d["modes"][key] and d["modes"][key]["value"] > 0, key


# ---- the overlap checks can fail (negative control) ---------------------------
@pytest.mark.parametrize("gather", ["rccl", "direct", "ipc"])
@pytest.mark.parametrize("chunks", ["1", "2"])
def test_two_ranks_overlap_check_catches_a_skipped_wait(gather, chunks, tmp_path):
    """matrix_parallel --overlap --check gives every unit its own product
    (B x 2^(k mod 3)) and checks each gathered piece of the last two units
    against its own unit: it PASSes as built and FAILs when the collectives are
    issued without their producer dependency (PDMB_TEST_SKIP_READY_WAIT), for
    the RCCL-shaped (here gloo), direct and ipc all-gathers, whole and
    signalled pieces (8192: two 256-workgroup rounds per shard GEMM)."""
    args = ["--sizes", "8192", "--iterations", "3", "--warmup", "1", "--mode", "matrix_parallel",
            "--overlap", "--chunks", chunks, "--check", "--allgather", gather]
    good = tmp_path / "good.jsonl"
    out = _run(2, "matmul_scaling_benchmark.py", *args, "--json", str(good))
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
    rec = _records(good)[-1]
    assert rec["plan"]["source"] == "measured"
    assert rec["signalled"] == (chunks == "2"), rec["plan"]
    assert len(rec["checked_units"]) == 2
    # the delay must outlast one gloo collective (tens of ms through the host):
    # a signalled unit's collective is issued behind the previous unit's, which
    # blocks this host thread under gloo, so a short delay would end first
    cycles = "20000000" if chunks == "1" else "800000000"
    out = _run(2, "matmul_scaling_benchmark.py", *args, env={"PDMB_TEST_SKIP_READY_WAIT": cycles})
    assert "FAIL" in out and "ERROR" not in out


@pytest.mark.parametrize("gather", ["rccl", "direct", "ipc"])
def test_eight_ranks_overlap_check_catches_a_skipped_wait(gather, tmp_path):
    """The negative control at ws = 8 (8 gloo ranks sharing the GPU): the same
    overlapped, checked matrix_parallel run FAILs its check when the collectives
    are issued without their producer dependency. (Its PASS half at ws = 8 is
    test_eight_ranks_scaling_overlap_checked.)"""
    args = ["--sizes", "4096", "--iterations", "3", "--warmup", "1", "--mode", "matrix_parallel",
            "--overlap", "--chunks", "1", "--check", "--allgather", gather]
    out = _run(8, "matmul_scaling_benchmark.py", *args, env={"PDMB_TEST_SKIP_READY_WAIT": "20000000"})
    assert "FAIL" in out and "ERROR" not in out


def test_eight_ranks_signalled_check_catches_a_skipped_wait():
    """ws = 8, signalled pieces (16384: the 16384 x 2048 shard GEMM spans two
    256-workgroup rounds, --chunks 2) through the ipc all-gather: without the
    producer dependency the check FAILs (its PASS half:
    test_eight_ranks_scaling_overlap_checked[matrix_parallel-16384-...])."""
    out = _run(8, "matmul_scaling_benchmark.py", "--sizes", "16384", "--iterations", "2", "--warmup", "1",
               "--mode", "matrix_parallel", "--overlap", "--chunks", "2", "--check", "--allgather", "ipc",
               env={"PDMB_TEST_SKIP_READY_WAIT": "800000000"})
    assert "FAIL" in out and "ERROR" not in out


# ---- the ws = 8 job shapes on real HIP (8 gloo ranks sharing the GPU) ---------
def _bench8(*extra, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--dist-backend", "gloo",
                        "--size", "4096", "--steps", "3", "--warmup", "1", "--extra-steps", "2",
                        "--extra-warmup", "1", *extra], cwd=ROOT, capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 8 and d["world_size_seen"] == 8 and d["value"] > 0
    assert d["collectives_verified"] is True and "modes_incomplete" not in d
    assert d["check"] == "pass", d["check_detail"]
    for key, m in d["modes"].items():
        assert m and "error" not in m and m["value"] > 0, (key, m)
        assert m["check"] == "pass", (key, m["check_detail"])  # Workload.verify, after timing
    return d


@pytest.mark.parametrize("extra,auto_ipc", [([], "0"), ([], "1"),
                                            (["--allgather", "ipc", "--allreduce", "ipc"], "0"),
                                            (["--mode", "matrix_parallel", "--overlap", "--chunks", "2",
                                              "--allgather", "ipc"], "0")])
def test_eight_ranks_self_launch_bench(extra, auto_ipc):
    """bench.py --gpus 8 through the self-launch path, the BASELINE ws = 8
    shapes (local batch 1 with a two-slot ring, 512-column shards at 4096):
    every mode runs, with measured overlap plans, and passes its check."""
    d = _bench8(*extra, env_extra={"PDMB_AUTO_IPC": auto_ipc})
    if not extra:  # auto on the overlapped modes: every candidate checked, then timed
        want = {"rccl", "direct", "ipc"} if auto_ipc == "1" else {"rccl", "direct"}
        colls = [m["collective"] for m in d["modes"].values() if m.get("collective")]
        assert colls and all(set(c["us"]) == want for c in colls), colls
        assert all(isinstance(v, float) for c in colls for v in c["us"].values()), colls
    plans = [m["plan"] for m in d["modes"].values() if m.get("plan")]
    plans += [d["config"]["overlap_plan"]] if "overlap_plan" in d["config"] else []
    assert plans and all(p["source"] == "measured" for p in plans), plans


@pytest.mark.parametrize("mode,size,extra", [
    ("matrix_parallel", "16384", ["--allgather", "ipc", "--chunks", "2"]),
    ("matrix_parallel", "4096", []),
    ("batch_parallel", "8192", ["--chunks", "2"]),
    ("batch_parallel", "8192", ["--allreduce", "ipc", "--chunks", "2"])])
def test_eight_ranks_scaling_overlap_checked(mode, size, extra, tmp_path):
    """matmul_scaling_benchmark.py at 8 ranks, overlapped and checked against
    float64: at 16384 / 8192 the unit GEMM spans two or more 256-workgroup
    rounds, so --chunks 2 runs signalled pieces; ipc maps all 7 peers."""
    js = tmp_path / "r.jsonl"
    out = _run(8, "matmul_scaling_benchmark.py", "--sizes", size, "--iterations", "2", "--warmup", "1",
               "--mode", mode, "--overlap", "--check", *extra, "--json", str(js))
    assert "Collective operations verified successfully across 8 GPUs" in out
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
    rec = _records(js)[-1]
    assert rec["plan"]["source"] == "measured"
    if "--chunks" in extra:
        assert rec["signalled"] is True and rec["pieces"] == 2, rec["plan"]
    if "ipc" in extra:
        assert rec["ipc_peers"] == 7


# ---- IPC register / close / free churn (VERDICT r4 "Next round" #1) -----------
@pytest.mark.parametrize("nproc", [2, 8])
@pytest.mark.parametrize("arena", ["0", "1"])
def test_ipc_churn_register_close_free(nproc, arena):
    """scripts/ipc_churn.py: 6 modes of allocate / register / all-gather +
    all-reduce (exact) / close / free, sizes alternating so freed buffers,
    handles and mappings are re-used — with the arena bypassed (the pre-arena
    behaviour, PDMB_IPC_ARENA=0) and with it — every pull bounds-checked on the
    host (PDMB_IPC_CHECK=1): every mode exact on every rank, no fault."""
    out = _run(nproc, "scripts/ipc_churn.py", "--modes", "6",
               env={"PDMB_IPC_ARENA": arena, "PDMB_IPC_CHECK": "1"})
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    modes = [r for r in recs if "mode" in r]
    assert len(modes) == 6 and all(r["all_gather_ok"] and r["all_reduce_ok"] for r in modes), recs
    assert all(r["arena"] == (arena == "1") and r["check"] for r in modes)
    if arena == "1":  # two sizes, two buffers each: the pool stops growing after mode 1
        assert modes[-1]["pool"][0] == 4 and modes[-1]["mapped"] == 4 * (nproc - 1), modes[-1]
    else:
        assert modes[-1]["pool"][0] == 0 and modes[-1]["mapped"] == 0
    assert recs[-1]["summary"] and recs[-1]["failed_modes"] == 0
