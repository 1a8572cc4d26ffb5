"""Reference-compatible function API (pytorch_distributed_matmul_benchmark_amd.api)."""
import torch

from pytorch_distributed_matmul_benchmark_amd import api


def test_signatures_and_returns_cpu():
    assert api.calculate_tflops(1000, 1.0) == 2e9 / 1e12
    t, tf = api.benchmark_matmul(128, torch.float32, "cpu", 2, 1)
    assert t > 0 and tf > 0
    t, tf = api.benchmark_independent(128, torch.float32, "cpu", 0, 2, 1)
    assert t > 0 and tf > 0
    t, tf = api.benchmark_batch_parallel(96, 4, torch.float32, "cpu", 0, 1, 2, 1)
    assert t > 0 and tf > 0
    t, tf = api.benchmark_matrix_parallel(96, torch.float32, "cpu", 0, 1, 2, 1)
    assert t > 0 and tf > 0
    t, tf = api.benchmark_ring_parallel(96, torch.float32, "cpu", 0, 1, 2, 1)
    assert t > 0 and tf > 0
    for f in (api.benchmark_data_parallel, api.benchmark_no_overlap, api.benchmark_overlap):
        t, tf, tc = f(96, torch.float32, "cpu", 0, 2, 1)
        assert t > 0 and tf > 0 and tc >= 0
    t, tf, tc = api.benchmark_pipeline(96, torch.float32, "cpu", 0, 3, 1, pipeline_depth=4)
    assert t > 0 and tf > 0
    t, tf, tc = api.benchmark_model_parallel(96, torch.float32, "cpu", 0, 1, 2, 1)
    assert t > 0 and tc == 0.0
    A, B = torch.randn(40, 30), torch.randn(30, 20)
    assert api.validate_result(A, B, A @ B) and not api.validate_result(A, B, A @ B * 1.1)
    assert api.ScalingMode.MATRIX_PARALLEL.value == "matrix_parallel"
    assert api.setup_distributed() == (0, 1)
    api.cleanup_distributed()
