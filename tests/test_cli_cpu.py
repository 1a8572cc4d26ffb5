"""CLI entry points end-to-end on CPU (BASELINE config #1: fp32 torch.matmul on CPU),
single process and under torchrun with gloo; output keeps the reference's
scraped substrings (backup/compare_benchmarks.py:22-26)."""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="2")


def _run(args, timeout=240):
    r = subprocess.run(args, cwd="/tmp", capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _torchrun(nproc, script, *args, port=None):
    port = port or free_port()
    return _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1",
                 f"--master-port={port}", os.path.join(ROOT, script), *args])


def test_basic_cpu_fp32(tmp_path):
    js = tmp_path / "r.jsonl"
    out = _run([sys.executable, os.path.join(ROOT, "matmul_benchmark.py"), "--device", "cpu",
                "--sizes", "256", "384", "--iterations", "2", "--warmup", "1",
                "--dtype", "float32", "--check", "--json", str(js)])
    for s in ("Results for 256x256", "Average time per multiplication", "TFLOPS per GPU",
              "Total TFLOPS (all GPUs)", "Required FLOPs per operation", "Benchmark completed!",
              "Check: max rel. error"):
        assert s in out, s
    assert "FAIL" not in out
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert [r["n"] for r in recs] == [256, 384]
    assert all(r["check_ok"] for r in recs)
    assert recs[0]["tflops_rank0"] > 0


@pytest.mark.parametrize("mode", ["independent", "batch_parallel", "matrix_parallel",
                                  "ring_parallel"])
def test_scaling_single_process(mode):
    out = _run([sys.executable, os.path.join(ROOT, "matmul_scaling_benchmark.py"), "--device",
                "cpu", "--sizes", "200", "--iterations", "2", "--warmup", "1", "--dtype",
                "float32", "--mode", mode, "--check"])
    assert "Actual TFLOPS (total FLOPs / time)" in out
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


@pytest.mark.parametrize("mode,extra", [("independent", []), ("batch_parallel", []),
                                        ("batch_parallel", ["--overlap", "--chunks", "2"]),
                                        ("matrix_parallel", []),
                                        ("matrix_parallel", ["--overlap", "--chunks", "3"])])
def test_scaling_torchrun_gloo(mode, extra, tmp_path):
    js = tmp_path / "r.jsonl"
    out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "300",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode", mode,
                    "--check", "--json", str(js), *extra)
    assert "Collective operations verified successfully across 2" in out
    assert "Results for 300x300" in out
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
    rec = json.loads(js.read_text().splitlines()[-1])
    assert rec["world_size"] == 2 and rec["mode"] == mode
    if mode == "batch_parallel":
        assert rec["global_batch"] == 4 and rec["local_batch"] == 2
    if mode == "matrix_parallel":
        assert rec["shard_cols"] == 152


@pytest.mark.parametrize("ws,n", [(2, 300), (3, 520)])
def test_ring_parallel_gloo(ws, n, tmp_path):
    """All-gather-GEMM over both ring directions: A row-sharded (512-row blocks,
    zero-padded; top halves travel clockwise, bottom halves counter-clockwise),
    each rank's C[:, S_r] checked against the float64 product of the global A."""
    js = tmp_path / "r.jsonl"
    out = _torchrun(ws, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", str(n),
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "ring_parallel", "--check", "--json", str(js))
    assert f"Results for {n}x{n}" in out
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
    rec = json.loads(js.read_text().splitlines()[-1])
    assert rec["mode"] == "ring_parallel" and rec["world_size"] == ws
    assert rec["hops"] == ws - 1 and rec["shard_rows"] == 512 and rec["directions"] == 2


@pytest.mark.parametrize("ws,mode,extra", [(4, "batch_parallel", ["--overlap", "--chunks", "2"]),
                                           (4, "matrix_parallel", ["--overlap", "--chunks", "2"]),
                                           (4, "ring_parallel", []),
                                           (8, "ring_parallel", [])])
def test_scaling_gloo_more_ranks(ws, mode, extra):
    """verify_collectives + float64-checked results at ws = 4 / 8."""
    out = _torchrun(ws, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "520",
                    "--iterations", "1", "--warmup", "1", "--dtype", "float32", "--mode", mode,
                    "--check", *extra)
    assert f"Collective operations verified successfully across {ws}" in out
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out


def test_batch_parallel_ws3_reports_real_batch(tmp_path):
    out = _torchrun(3, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "128",
                    "--iterations", "1", "--warmup", "1", "--dtype", "float32", "--mode",
                    "batch_parallel", "--check")
    assert "Processing 6 total batches across 3 GPU(s) (2 per GPU)" in out
    assert "PASS" in out


@pytest.mark.parametrize("mode", ["independent", "data_parallel", "model_parallel"])
def test_backup_distributed(mode):
    out = _torchrun(2, "backup/matmul_distributed_benchmark.py", "--device", "cpu", "--sizes",
                    "256", "--iterations", "2", "--warmup", "1", "--mode", mode, "--check",
                    )
    assert "Total time per operation" in out and "PASS" in out and "ERROR" not in out
    if mode != "independent":
        assert "Communication overhead" in out


@pytest.mark.parametrize("mode", ["no_overlap", "overlap", "pipeline"])
def test_backup_overlap(mode):
    out = _torchrun(2, "backup/matmul_overlap_benchmark.py", "--device", "cpu", "--sizes", "256",
                    "--iterations", "3", "--warmup", "1", "--mode", mode, "--check")
    assert "Actual TFLOPS" in out and "Compute-only TFLOPS" in out
    assert "PASS" in out and "ERROR" not in out


def test_compare_benchmarks_any_cwd():
    out = _run([sys.executable, os.path.join(ROOT, "backup", "compare_benchmarks.py"), "--gpus",
                "2", "--dtype", "float32", "--size", "128", "--extra",
                "--device cpu --sizes 128 --iterations 1 --warmup 1"], timeout=400)
    assert out.count("Results for 128x128") == 4
    assert "FAILED" not in out


def test_launcher_single_process():
    out = _run(["bash", os.path.join(ROOT, "run_scaling_benchmark.sh"), "1", "matrix_parallel",
                "float32", "--device", "cpu", "--sizes", "128", "--iterations", "1",
                "--warmup", "1"])
    assert "Running in single GPU mode" in out and "Results for 128x128" in out


def test_resume_skips_recorded_sizes(tmp_path):
    js = tmp_path / "r.jsonl"
    args = [sys.executable, os.path.join(ROOT, "matmul_scaling_benchmark.py"), "--device", "cpu",
            "--iterations", "1", "--warmup", "0", "--dtype", "float32", "--json", str(js)]
    _run(args + ["--sizes", "64"])
    out = _run(args + ["--sizes", "64", "96", "--resume"])
    assert "Skipping 64x64" in out and "Results for 96x96" in out
    assert len(js.read_text().splitlines()) == 2


def test_mode_enums_and_validate_result():
    import torch

    from pytorch_distributed_matmul_benchmark_amd.models import (BenchmarkMode, ScalingMode,
                                                                 Workload, run_mode)
    from pytorch_distributed_matmul_benchmark_amd.models.common import validate_result
    from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

    assert [m.value for m in ScalingMode] == ["independent", "batch_parallel", "matrix_parallel"]
    assert BenchmarkMode("pipeline") is BenchmarkMode.PIPELINE
    r = run_mode(ScalingMode.BATCH_PARALLEL,
                 Workload(n=64, dtype=torch.float32, iters=1, warmup=0, check=True), DistContext())
    assert r.relerr < 1e-5 and r.extra["global_batch"] == 4
    A, B = torch.randn(70, 33), torch.randn(33, 20)
    assert validate_result(A, B, A @ B) and not validate_result(A, B, A @ B + 0.1)


def test_scaling_ref_reports_efficiency_vs_one_rank(tmp_path):
    js = tmp_path / "r.jsonl"
    out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "160",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "independent", "--scaling-ref", "--json", str(js))
    assert "Scaling efficiency vs 1 GPU:" in out
    rec = json.loads(js.read_text().splitlines()[-1])
    assert rec["single_gpu_tflops"] > 0 and rec["scaling_efficiency_vs_1gpu"] > 0


def test_fp8_cli_cpu_and_gloo(tmp_path):
    """--dtype float8_e4m3fn end to end: e4m3 operands (B column-major), bf16 C, float64
    check of the same quantized values; single process and 2 gloo ranks with overlap."""
    out = _run([sys.executable, os.path.join(ROOT, "matmul_benchmark.py"), "--device", "cpu",
                "--sizes", "256", "--iterations", "2", "--warmup", "1",
                "--dtype", "float8_e4m3fn", "--check"])
    assert "Check: max rel. error" in out and "PASS" in out and "FAIL" not in out
    for mode in ("batch_parallel", "matrix_parallel"):
        out = _torchrun(2, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "300",
                        "--iterations", "2", "--warmup", "1", "--dtype", "float8_e4m3fn",
                        "--mode", mode, "--overlap", "--chunks", "2", "--check")
        assert out.count("PASS") == 1 and "FAIL" not in out and "ERROR" not in out


@pytest.mark.parametrize("ws,extra", [(2, []), (3, ["--overlap", "--chunks", "2"]),
                                      (4, ["--overlap", "--chunks", "3"])])
def test_matrix_parallel_direct_allgather(ws, extra):
    """--allgather direct: the shard goes to every peer in one batched P2P group
    (each over its own link on a fully connected node); the gathered C is checked
    against the float64 product, serialized and overlapped."""
    out = _torchrun(ws, "matmul_scaling_benchmark.py", "--device", "cpu", "--sizes", "300",
                    "--iterations", "2", "--warmup", "1", "--dtype", "float32", "--mode",
                    "matrix_parallel", "--allgather", "direct", "--check", *extra)
    assert "PASS" in out and "FAIL" not in out and "ERROR" not in out
