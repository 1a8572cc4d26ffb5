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
