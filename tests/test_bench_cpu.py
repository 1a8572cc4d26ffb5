"""bench.py's driver contract on the multi-rank path (torchrun + gloo on CPU):
one JSON line from rank 0 with the required keys, whole-job value, max-over-ranks time."""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def _bench(nproc, *args, port=None):
    port = port or free_port()
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
                        f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--gpus", str(nproc), *args], capture_output=True, text=True, timeout=300,
                       cwd="/tmp", env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("mode,extra,scaling,gb", [
    ("independent", [], "weak", 2), ("batch_parallel", [], "weak", 4),
    ("batch_parallel", ["--overlap"], "weak", 4), ("matrix_parallel", [], "strong", 1),
    ("matrix_parallel", ["--overlap", "--chunks", "2"], "strong", 1)])
def test_bench_two_ranks(mode, extra, scaling, gb):
    d = _bench(2, "--size", "256", "--steps", "3", "--warmup", "1", "--mode", mode, *extra)
    for k in KEYS:
        assert k in d, k
    if "--overlap" in extra:
        assert d["config"]["overlap_plan"]["source"] == "measured"
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["scaling"] == scaling and d["config"]["global_batch"] == gb
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["vs_baseline"] is None  # CPU / non-16k runs are never compared to the reference
    # value is the whole-job aggregate: FLOPs of all ranks / max-over-ranks time
    flops = 2.0 * 256 ** 3 * (2 if mode == "independent" else gb)
    assert d["value"] == pytest.approx(flops / (d["ms_per_step"] / 1e3) / 1e12, rel=0.02, abs=1e-4)


@pytest.mark.parametrize("nproc", [2, 3])
def test_bench_ring_parallel_opt_in(nproc):
    d = _bench(nproc, "--size", "256", "--steps", "2", "--warmup", "1", "--mode", "ring_parallel",
               "--extra-steps", "0")
    assert d["config"]["parallelism"] == f"ring{nproc}" and d["scaling"] == "strong"
    assert d["value"] == pytest.approx(2.0 * 256 ** 3 / (d["ms_per_step"] / 1e3) / 1e12,
                                       rel=0.02, abs=1e-4)
    assert d["vs_baseline"] is None and d["modes"] == {}


def test_bench_four_ranks_batch_never_empty():
    d = _bench(4, "--size", "128", "--steps", "2", "--warmup", "1", "--mode", "batch_parallel",
               )
    assert d["config"]["global_batch"] == 4 and d["config"]["parallelism"] == "dp4"


def test_bench_reports_secondary_modes():
    """The headline line also carries batch_parallel / matrix_parallel (serialized and
    overlapped) timed in the same job, each with its own whole-job value."""
    d = _bench(2, "--size", "256", "--steps", "2", "--warmup", "1", "--extra-steps", "2",
               "--extra-warmup", "1")
    assert set(d["modes"]) == {"batch_parallel", "batch_parallel+overlap", "matrix_parallel",
                               "matrix_parallel+overlap"}
    for key, m in d["modes"].items():
        assert m["value"] > 0 and m["ms_per_step"] > 0 and m["steps"] == 2
        gb = 4 if key.startswith("batch") else 1
        assert m["global_batch"] == gb
        assert m["parallelism"] == ("dp2" if gb == 4 else "tp2")
        assert m["value"] == pytest.approx(2.0 * 256 ** 3 * gb / (m["ms_per_step"] / 1e3) / 1e12,
                                           rel=0.02, abs=1e-4)
    assert d["config"]["mode"] == "independent"
    d0 = _bench(2, "--size", "128", "--steps", "1", "--warmup", "0", "--extra-steps", "0",
                "--mode", "batch_parallel")
    assert d0["modes"] == {}


def test_bench_eight_ranks_driver_form():
    """The driver's N = 8 launch (torchrun --nproc-per-node 8 ... bench.py --gpus 8)
    rehearsed on gloo: every secondary mode, serialized and overlapped, runs at
    ws = 8 with its agreed plan; batch_parallel's global batch is rounded up to
    one element per rank, matrix_parallel shards 8 ways."""
    d = _bench(8, "--size", "128", "--steps", "2", "--warmup", "1", "--extra-steps", "1",
               "--extra-warmup", "0")
    assert d["n_gpus"] == 8 and d["world_size_seen"] == 8 and d["collectives_verified"] is True
    assert d["config"]["parallelism"] == "independent8" and d["scaling_efficiency"] is not None
    assert set(d["modes"]) == {"batch_parallel", "batch_parallel+overlap", "matrix_parallel",
                               "matrix_parallel+overlap"}
    assert d["check"] == "pass", d["check_detail"]
    for key, m in d["modes"].items():
        assert "error" not in m, (key, m)
        # every mode's last step checked after its timed region (Workload.verify)
        assert m["check"] == "pass", (key, m["check_detail"])
        if key.endswith("+overlap"):
            c = m["collective"]  # every auto candidate passed the payload gate and was timed
            assert all(isinstance(v, float) for v in c["us"].values()), c
        gb = 8 if key.startswith("batch") else 1
        assert m["global_batch"] == gb and m["parallelism"] == ("dp8" if gb == 8 else "tp8")
        assert m["value"] == pytest.approx(2.0 * 128 ** 3 * gb / (m["ms_per_step"] / 1e3) / 1e12,
                                           rel=0.02, abs=1e-4)
        if key.endswith("+overlap"):
            # priced from the job's own measured GEMM / collective times (MAX over ranks)
            plan = m["plan"]
            assert plan["source"] == "measured", (key, plan)
            assert plan["comm_us"] == plan["piece_us"]["1"] > 0 and plan["gemm_us"] > 0
            assert plan["serial_us"] == pytest.approx(plan["gemm_us"] + plan["comm_us"], abs=0.2)


def _plain(*args, env_extra=None, timeout=300):
    """bench.py run WITHOUT torchrun (the driver's 1-GPU form; --gpus N self-launches)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                           *args], capture_output=True, text=True, timeout=timeout, cwd="/tmp",
                          env=env)


def _line(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    return json.loads(lines[0])


def test_bench_self_launches_n_ranks():
    """--gpus 4 with no torchrun: bench.py starts 4 ranks itself, one JSON line,
    whole-job value, and an in-job scaling efficiency vs rank 0 alone."""
    r = _plain("--gpus", "4", "--size", "256", "--steps", "3", "--warmup", "1",
               "--extra-steps", "1", "--extra-warmup", "0")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r)
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "independent4"
    assert d["single_gpu_tflops"] > 0
    # value / single / efficiency are each rounded to 4 places, and on the CPU at this size
    # the TFLOPS fields are ~1e-3, so bound the efficiency by the rounding interval instead
    # of a relative tolerance.
    v, s, h = d["value"], d["single_gpu_tflops"], 5e-5
    lo, hi = (v - h) / (4 * (s + h)), (v + h) / (4 * max(s - h, 1e-12))
    assert lo - h <= d["scaling_efficiency"] <= hi + h, (d["scaling_efficiency"], lo, hi)
    for key, m in d["modes"].items():
        assert m["scaling_efficiency"] is not None, key


def test_bench_ws1_overlap_modes_are_null():
    d = _line(_plain("--size", "128", "--steps", "1", "--warmup", "0", "--extra-steps", "1",
                     "--extra-warmup", "0"))
    assert d["n_gpus"] == 1 and d["scaling_efficiency"] == 1.0
    assert d["modes"]["batch_parallel+overlap"] is None
    assert d["modes"]["matrix_parallel+overlap"] is None
    assert d["modes"]["batch_parallel"]["value"] > 0


def test_bench_world_size_mismatch_is_an_error():
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--gpus", "4", "--size", "64"], capture_output=True, text=True,
                       timeout=120, cwd="/tmp", env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_bench_refuses_test_fault_injection():
    """A PDMB_TEST_* negative-control switch (racy collectives) never yields a
    driver line (such a run must not pass for a measurement)."""
    env = dict(os.environ, PDMB_TEST_SKIP_READY_WAIT="1000")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--size", "64", "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, timeout=120, cwd="/tmp", env=env)
    assert r.returncode == 2 and "PDMB_TEST_SKIP_READY_WAIT" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_setup_failure_on_one_rank_is_agreed():
    """A secondary mode that fails to set up on rank 1 only becomes an "error"
    entry on rank 0's line; the headline and the other modes still report."""
    r = _plain("--gpus", "2", "--size", "128", "--steps", "1", "--warmup", "0",
               "--extra-steps", "1", "--extra-warmup", "0",
               env_extra={"PDMB_BENCH_FAULT": "1:matrix_parallel:setup"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r)
    assert "error" in d["modes"]["matrix_parallel"]
    assert d["modes"]["batch_parallel"]["value"] > 0 and d["value"] > 0


@pytest.mark.parametrize("spec", ["1:batch_parallel:timed", "1:independent:setup"])
def test_bench_fault_exits_fast(spec):
    """A timed-region fault on one rank (peers blocked in a collective) or a failed
    headline ends the whole job non-zero within seconds, not at the PG timeout."""
    import time

    t0 = time.time()
    r = _plain("--gpus", "2", "--size", "128", "--steps", "2", "--warmup", "1",
               "--extra-steps", "2", "--extra-warmup", "1",
               env_extra={"PDMB_BENCH_FAULT": spec, "PDMB_PG_TIMEOUT": "600"}, timeout=240)
    assert r.returncode != 0
    assert time.time() - t0 < 90
    assert "injected fault" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if spec.endswith("setup"):  # the headline itself failed: no line
        assert lines == []
    else:  # a secondary mode died after the headline: rank 0 still prints it
        assert len(lines) == 1, r.stdout
        d = json.loads(lines[0])
        assert d["value"] > 0 and "modes_incomplete" in d
        assert "batch_parallel" not in d["modes"]


@pytest.mark.parametrize("spec", ["0:matrix_parallel:timed", "1:matrix_parallel+overlap:timed"])
def test_bench_headline_survives_a_secondary_mode_death(spec):
    """A timed-region death in a secondary mode, on rank 0 itself (``_die``) or on
    another rank (torchrun's SIGTERM reaches rank 0 while it is blocked in a
    collective): rank 0's one line still carries the headline and the modes that
    finished, plus ``modes_incomplete``; the job still exits non-zero."""
    r = _plain("--gpus", "2", "--size", "128", "--steps", "2", "--warmup", "1",
               "--extra-steps", "2", "--extra-warmup", "1",
               env_extra={"PDMB_BENCH_FAULT": spec, "PDMB_PG_TIMEOUT": "600"}, timeout=240)
    assert r.returncode != 0
    d = _line(r)
    assert d["value"] > 0 and d["n_gpus"] == 2
    assert d["modes"]["batch_parallel"]["value"] > 0  # finished before the fault
    assert "matrix_parallel" in d["modes_incomplete"] or "signal" in d["modes_incomplete"]


_NO_HIP = """
import runpy, sys, torch
sys.path.insert(0, {root!r})
def boom(*a, **k):
    raise RuntimeError("the self-launch parent touched HIP")
torch._C._cuda_getDeviceCount = boom
torch.cuda.device_count = boom
torch.cuda.is_available = boom
{extra}
sys.argv = ["bench.py"] + {args!r}
runpy.run_path({path!r}, run_name="__main__")
"""


def _parent_without_hip(args, extra=""):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    code = _NO_HIP.format(extra=extra, args=list(args), path=os.path.join(ROOT, "bench.py"), root=ROOT)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                          cwd="/tmp", env=env)


def test_self_launch_parent_never_counts_gpus_through_hip():
    """The --gpus N parent counts GPUs from sysfs / amdsmi only (utils/telemetry.py):
    with HIP's device count patched to raise it still self-launches 4 ranks, and
    on a box with too few GPUs it refuses with rc 2 at once."""
    r = _parent_without_hip(["--device", "cpu", "--gpus", "4", "--size", "128", "--steps", "1",
                             "--warmup", "0", "--extra-steps", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert _line(r)["n_gpus"] == 4
    r = _parent_without_hip(["--gpus", "2", "--size", "128"],
                            extra="import pytorch_distributed_matmul_benchmark_amd.utils.telemetry as t;"
                                  " t.visible_gpus = lambda: 1")
    assert r.returncode == 2 and "only 1 GPU" in r.stderr, r.stderr[-2000:]


def test_bench_json_verifiability_fields():
    """ws = 1 (no process group) and ws = 2 (gloo) lines carry every field the
    driver needs to check a multi-GPU run: backend, world size the group saw,
    RCCL version, collective self-test, per-rank TFLOPS, per-mode split / plan /
    warm-up and the rank-0-alone references."""
    keys = ("dist_backend", "world_size_seen", "rccl_version", "collectives_verified",
            "per_rank_tflops", "sclk_mhz", "power_w")
    d1 = _line(_plain("--size", "128", "--steps", "1", "--warmup", "0", "--extra-steps", "1",
                      "--extra-warmup", "0"))
    assert all(k in d1 for k in keys)
    assert d1["world_size_seen"] == 1 and d1["dist_backend"] is None
    d2 = _bench(2, "--size", "128", "--steps", "1", "--warmup", "0", "--extra-steps", "1",
                "--extra-warmup", "0", "--chunks", "1")
    assert d2["dist_backend"] == "gloo" and d2["world_size_seen"] == 2
    assert d2["collectives_verified"] is True
    assert d2["per_rank_tflops"]["min"] <= d2["per_rank_tflops"]["max"]
    for key in ("batch_parallel", "matrix_parallel"):
        m = d2["modes"][key]
        assert m["compute_ms"] >= 0 and m["comm_ms"] >= 0 and "warmup_ms" in m
        assert m["ref_tflops_rank0_alone"] > 0 and m["scaling_efficiency"] is not None
    assert d2["modes"]["batch_parallel+overlap"]["plan"]["overlap"] is True  # --chunks 1: requested


def test_bench_secondary_deadline_prints_the_headline():
    """Secondary modes that outlive --extra-deadline-s (a stuck collective): rank 0
    prints its line with modes_incomplete and the job ends, well before the
    process-group timeout."""
    import time

    t0 = time.time()
    r = _plain("--gpus", "2", "--size", "256", "--steps", "2", "--warmup", "1",
               "--extra-steps", "20000", "--extra-warmup", "1", "--extra-deadline-s", "3",
               env_extra={"PDMB_PG_TIMEOUT": "600"}, timeout=240)
    assert time.time() - t0 < 120
    d = _line(r)
    assert d["value"] > 0 and "after 3 s" in d["modes_incomplete"]
    assert r.returncode != 0
