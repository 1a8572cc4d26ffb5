"""The Python-free native executor (runtime/pdmb_bench: HIP threads + RCCL) on the GPU:
every scaling mode, serialized and overlapped, with the float64 end-to-end check."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "pytorch_distributed_matmul_benchmark_amd", "runtime", "pdmb_bench")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        from pytorch_distributed_matmul_benchmark_amd.ops import build
        build.build_bench()
    return EXE


@pytest.mark.parametrize("mode,extra", [("independent", []), ("batch_parallel", []),
                                        ("batch_parallel", ["--overlap"]),
                                        ("matrix_parallel", []),
                                        ("matrix_parallel", ["--overlap"]),
                                        ("matrix_parallel", ["--allgather", "direct"]),
                                        ("matrix_parallel", ["--overlap", "--allgather", "direct"]),
                                        ("matrix_parallel", ["--allgather", "ipc"]),
                                        ("matrix_parallel", ["--overlap", "--allgather", "ipc"]),
                                        ("batch_parallel", ["--allreduce", "ipc"]),
                                        ("batch_parallel", ["--overlap", "--allreduce", "ipc"]),
                                        ("batch_parallel", ["--allreduce", "direct"]),
                                        ("batch_parallel", ["--overlap", "--allreduce", "direct"]),
                                        ("ring_parallel", [])])
@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_native_executor_modes(exe, mode, extra, dtype, tmp_path):
    js = tmp_path / "r.jsonl"
    r = subprocess.run([exe, "--gpus", "1", "--sizes", "1024", "2304", "--iterations", "3",
                        "--warmup", "1", "--dtype", dtype, "--mode", mode, "--check",
                        "--json", str(js), *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("PASS") == 2 and "FAIL" not in r.stdout
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert [x["n"] for x in recs] == [1024, 2304]
    assert all(x["node_tflops"] > 0 and x["relerr"] is not None for x in recs)


@pytest.mark.parametrize("mode,extra", [("independent", []), ("batch_parallel", []),
                                        ("batch_parallel", ["--overlap"]),
                                        ("matrix_parallel", []),
                                        ("matrix_parallel", ["--overlap"]),
                                        ("ring_parallel", [])])
def test_native_executor_fp8(exe, mode, extra, tmp_path):
    """--dtype float8_e4m3fn: e4m3 operands (B column-major, its column shard a
    row range of Bt), bf16 C through the collectives, float64 check of the
    decoded operands."""
    js = tmp_path / "r.jsonl"
    r = subprocess.run([exe, "--gpus", "1", "--sizes", "1024", "2304", "--iterations", "3",
                        "--warmup", "1", "--dtype", "float8_e4m3fn", "--mode", mode, "--check",
                        "--json", str(js), *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("PASS") == 2 and "FAIL" not in r.stdout
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert all(x["dtype"] == "float8_e4m3fn" and x["relerr"] < 1e-2 for x in recs)
    assert all(x["kernel"].startswith("pdmb_fp8") for x in recs), recs


@pytest.mark.parametrize("mode", ["batch_parallel", "matrix_parallel"])
def test_native_executor_signalled_overlap(exe, mode, tmp_path):
    """--overlap --chunks 2 at 8192: the W4 GEMM signals each 4096-row piece and the
    rank thread issues that piece's RCCL collective while the launch still runs."""
    js = tmp_path / "r.jsonl"
    r = subprocess.run([exe, "--gpus", "1", "--sizes", "8192", "--iterations", "4", "--warmup", "2",
                        "--mode", mode, "--overlap", "--chunks", "2", "--check", "--json", str(js),
                        *(["--batch", "1"] if mode == "batch_parallel" else [])],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("PASS") == 1 and "FAIL" not in r.stdout
    rec = json.loads(js.read_text().splitlines()[0])
    assert rec["pieces"] == 2 and rec["relerr"] < 1e-2
