"""GPU integration: every mode on the native kernels with end-to-end checks,
RCCL bring-up under torchrun, bench.py's JSON contract and the smoke hook."""
import json
import os
import subprocess
import sys

import pytest
from conftest import free_port
import torch

from pytorch_distributed_matmul_benchmark_amd.models import MODES, Workload, run_mode
from pytorch_distributed_matmul_benchmark_amd.models.common import tolerance
from pytorch_distributed_matmul_benchmark_amd.parallel.dist import DistContext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ctx():
    return DistContext(rank=0, world_size=1, local_rank=0, device=torch.device("cuda", 0))


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float8_e4m3fn])
def test_mode_single_gpu(mode, dtype):
    w = Workload(n=1024, dtype=dtype, iters=3, warmup=1, check=True, batch=2)
    r = run_mode(mode, w, _ctx())
    assert r.relerr is not None and r.relerr < tolerance(dtype), r.relerr
    assert r.avg_ms > 0 and r.tflops > 0
    assert r.kernel.startswith("pdmb_fp8" if dtype == torch.float8_e4m3fn else ("pdmb_w4", "pdmb_t1", "pdmb_t2", "pdmb_mfma256"))


def test_fp32_independent_uses_exact_mfma():
    w = Workload(n=512, dtype=torch.float32, iters=2, warmup=1, check=True)
    r = run_mode("independent", w, _ctx())
    assert r.kernel.startswith("pdmb_f32_") and r.relerr < tolerance(torch.float32)


def test_graph_replay_independent():
    w = Workload(n=2048, iters=5, warmup=1, check=True, graph=True)
    r = run_mode("independent", w, _ctx())
    assert r.relerr < tolerance(torch.bfloat16)


def test_native_vs_torch_backend_agree():
    torch.manual_seed(0)
    A = torch.randn(768, 1280, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(1280, 1536, device="cuda", dtype=torch.bfloat16)
    from pytorch_distributed_matmul_benchmark_amd.ops import gemm
    C = gemm.matmul(A, B)
    R = torch.matmul(A.float(), B.float())
    assert ((C.float() - R).norm() / R.norm()).item() < 5e-3


def _run(args, timeout=400):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("mode,extra", [("independent", []), ("batch_parallel", []),
                                        ("batch_parallel", ["--overlap"]),
                                        ("matrix_parallel", [])])
def test_torchrun_rccl_single_rank(mode, extra):
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                "--master-addr=127.0.0.1", f"--master-port={free_port()}", "matmul_scaling_benchmark.py",
                "--sizes", "1024", "2048", "--iterations", "3", "--warmup", "1", "--mode", mode,
                "--check", *extra])
    assert "Results for 2048x2048" in out and "PASS" in out
    assert "FAIL" not in out and "ERROR" not in out
    assert any(k in out for k in ("pdmb_w4_nn", "pdmb_w4s", "pdmb_t128", "pdmb_t256x128", "pdmb_t192",
                                 "pdmb_mfma256"))


def test_bench_json_contract():
    out = _run([sys.executable, "bench.py", "--size", "2048", "--steps", "4", "--warmup", "1"])
    line = [l for l in out.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["value"] > 0
    assert d["config"]["kernel"].startswith(("pdmb_w4", "pdmb_t1", "pdmb_t2"))  # 2048^3: a small tile


def test_smoke_hook():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    ge.smoke()


def test_autograd_batched_broadcast():
    from pytorch_distributed_matmul_benchmark_amd.ops.autograd import native_matmul
    torch.manual_seed(5)
    A = torch.randn(2, 256, 320, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    B = torch.randn(320, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    native_matmul(A, B).float().sum().backward()
    Ar, Br = A.detach().double().requires_grad_(), B.detach().double().requires_grad_()
    (Ar @ Br).sum().backward()
    for g, r in ((A.grad, Ar.grad), (B.grad, Br.grad)):
        assert ((g.double() - r).norm() / r.norm()).item() < 1e-2


def test_reference_function_api_on_gpu():
    from pytorch_distributed_matmul_benchmark_amd import api
    t, tf = api.benchmark_matmul(2048, torch.bfloat16, "cuda:0", 5, 2)
    assert t > 0 and tf > 100
    t, tf, tc = api.benchmark_pipeline(1024, torch.bfloat16, "cuda:0", 0, 4, 1, pipeline_depth=3)
    assert t > 0 and tf > 0
