"""CU-masked compute streams (parallel/overlap.py MaskedStream): the mask is what
was asked for, and the native GEMMs are exact on such a stream."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import gemm
from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import MaskedStream, compute_stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [8, 32])
def test_masked_stream_excludes_k_cus_and_gemm_is_exact(k):
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ms = MaskedStream(dev, k)
    try:
        assert ms.active_cus() == ncu - k
        g = torch.Generator(device="cuda").manual_seed(k)
        A = torch.randint(-3, 4, (4096, 2048), device="cuda", generator=g).to(torch.bfloat16)
        B = torch.randint(-3, 4, (2048, 2048), device="cuda", generator=g).to(torch.bfloat16)
        with torch.cuda.stream(ms.stream):
            C = gemm.matmul(A, B)
            C2 = gemm.matmul(A[:1024], B, splitk=2, kernel="t128")
        torch.cuda.current_stream().wait_stream(ms.stream)
        torch.cuda.synchronize()
        R = (A.double() @ B.double()).to(torch.bfloat16)
        assert torch.equal(C, R) and torch.equal(C2, R[:1024])
    finally:
        ms.close()


def test_compute_stream_without_mask_is_current():
    dev = torch.device("cuda", 0)
    s, owner = compute_stream(dev, 0)
    assert owner is None and s == torch.cuda.current_stream(dev)


@pytest.mark.parametrize("k", [8, 32])
@pytest.mark.parametrize("kernel", ["auto", "w4", "w4s"])
def test_budgeted_gemm_on_masked_stream_is_exact(k, kernel):
    """GEMMs planned for the CU budget of a masked stream (ops.gemm.cu_budget:
    W4 with its budget-sized split / grid, W4S with G = 256 - k workgroups) on the
    ws = 8 shard's tile grid (64 x 8 tiles of 256^2 on 248 / 224 CUs) are exact."""
    dev = torch.device("cuda", 0)
    ms = MaskedStream(dev, k)
    try:
        g = torch.Generator(device="cuda").manual_seed(100 + k)
        A = torch.randint(-3, 4, (16384, 1024), device="cuda", generator=g).to(torch.bfloat16)
        B = torch.randint(-3, 4, (1024, 2048), device="cuda", generator=g).to(torch.bfloat16)
        R = (A.double() @ B.double()).to(torch.bfloat16)
        with torch.cuda.stream(ms.stream), ms.budget():
            C = gemm.matmul(A, B, kernel=kernel)
        torch.cuda.current_stream().wait_stream(ms.stream)
        torch.cuda.synchronize()
        assert torch.equal(C, R)
    finally:
        ms.close()
