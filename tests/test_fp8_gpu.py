"""fp8 (OCP e4m3fn) GEMM on the block-scaled MFMA (gemm_fp8.hip) vs a float64
reference of the same dequantized operands. bf16 output: exact-integer cases
compare bit-for-bit after rounding the fp64 reference to bf16."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import gemm

pytestmark = pytest.mark.gpu
FP8 = torch.float8_e4m3fn
FP8_KERNELS = ("pdmb_fp8_w4_nt", "pdmb_fp8_w4s", "pdmb_fp8_t128_nt", "pdmb_fp8_t256x128_nt",
               "pdmb_fp8_t192_nt", "pdmb_fp8_t192x128_nt")


def _ints(shape, g, lo=-3, hi=4):
    return torch.randint(lo, hi, shape, device="cuda", generator=g).float()


def _colmajor(x):
    """[K,N] view of a row-major [N,K] copy (the fp8 B layout)."""
    return x.transpose(-1, -2).contiguous().transpose(-1, -2)


def _relerr(x, ref):
    return ((x.double() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 256), (1000, 1052, 384),
                                   (300, 200, 128), (2304, 2048, 1024), (256, 512, 256),
                                   (768, 256, 640),
                                   (2048, 8192, 256), (8192, 2048, 256)])  # thin-grid super-tiles
def test_fp8_exact_small_integers(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + K)
    Af, Bf = _ints((M, K), g), _ints((K, N), g)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    assert gemm.kernel_for(A8, B8) in FP8_KERNELS
    ref = (Af.double() @ Bf.double()).to(torch.bfloat16)
    C = gemm.matmul(A8, B8)
    assert C.dtype == torch.bfloat16 and C.shape == (M, N)
    assert torch.equal(C, ref)
    C = gemm.matmul(A8, B8, kernel="fp8_w4")  # W4 handles every shape (edge tiles)
    assert torch.equal(C, ref)


def test_fp8_identity_with_asymmetric_b():
    n = 512
    A = torch.eye(n, device="cuda")
    B = ((torch.arange(n * n, device="cuda").view(n, n) * 7) % 13 - 6).float()  # asymmetric
    C = gemm.matmul(A.to(FP8), _colmajor(B.to(FP8)))
    assert torch.equal(C.float(), B)
    C = gemm.matmul(B.to(FP8), _colmajor(A.to(FP8)))
    assert torch.equal(C.float(), B)


def test_fp8_row_major_b_is_accepted():
    g = torch.Generator(device="cuda").manual_seed(5)
    Af, Bf = _ints((512, 256), g), _ints((256, 384), g)
    C = gemm.matmul(Af.to(FP8), Bf.to(FP8))  # row-major B: copied to column-major
    assert torch.equal(C, (Af.double() @ Bf.double()).to(torch.bfloat16))


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (1536, 1280, 2048)])
def test_fp8_random_scaled(M, N, K):
    torch.manual_seed(M + N)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(K, N, device="cuda")
    A8, sa = gemm.fp8_quantize(A)
    B8, sb = gemm.fp8_quantize(B, colmajor=True)
    assert B8.stride(-2) == 1
    C = gemm.matmul(A8, B8, alpha=sa * sb)
    ref = (A8.double() * sa) @ (B8.double() * sb)  # same quantized operands
    assert _relerr(C, ref) < 8e-3  # bf16 output rounding
    assert _relerr(C, A.double() @ B.double()) < 8e-2  # vs unquantized: e4m3 error


def test_fp8_batched_and_column_shards():
    g = torch.Generator(device="cuda").manual_seed(3)
    Af, Bf = _ints((3, 384, 256), g), _ints((3, 256, 640), g)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    C = gemm.matmul(A8, B8)
    assert torch.equal(C, torch.bmm(Af.double(), Bf.double()).to(torch.bfloat16))
    # matrix_parallel-style column shards of a column-major B are row slices of Bt
    Bt = _ints((1024, 512), g).to(FP8)  # [N, K]
    Ai = _ints((640, 512), g)
    for r in range(4):
        Bs = Bt[r * 256:(r + 1) * 256].t()  # [K, 256] column-major view, no copy
        assert Bs.stride(-2) == 1
        C = gemm.matmul(Ai.to(FP8), Bs)
        ref = (Ai.double() @ Bs.double()).to(torch.bfloat16)
        assert torch.equal(C, ref)


@pytest.mark.parametrize("kernel", ["fp8_w4", "fp8"])
def test_fp8_race_screen(kernel):
    if kernel in gemm.EXPERIMENT_KERNELS and not gemm.experiments_built():
        pytest.skip("8-wave fp8 kernel: PDMB_EXPERIMENTS=1 build only")
    torch.manual_seed(11)
    A8, sa = gemm.fp8_quantize(torch.randn(4096, 4096, device="cuda"))
    B8, sb = gemm.fp8_quantize(torch.randn(4096, 4096, device="cuda"), colmajor=True)
    ref = gemm.matmul(A8, B8, alpha=sa * sb, kernel=kernel)
    assert _relerr(ref, (A8.double() * sa) @ (B8.double() * sb)) < 8e-3
    for _ in range(20):
        assert torch.equal(gemm.matmul(A8, B8, alpha=sa * sb, kernel=kernel), ref)


@pytest.mark.experiments
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (1000, 1052, 384), (2304, 2048, 1024),
                                   (512, 512, 384)])
def test_fp8_8wave_kernel_exact(M, N, K):
    """The 8-wave SCHED-3 fp8 kernel (kept for A/B) on the exact-integer cases."""
    if not gemm.experiments_built():
        pytest.skip("8-wave fp8 kernel: PDMB_EXPERIMENTS=1 build only")
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    Af, Bf = _ints((M, K), g), _ints((K, N), g)
    C = gemm.matmul(Af.to(FP8), _colmajor(Bf.to(FP8)), kernel="fp8")
    assert torch.equal(C, (Af.double() @ Bf.double()).to(torch.bfloat16))


def test_fp8_unsupported_shape_fails_loudly():
    A8 = torch.zeros(256, 96, device="cuda").to(FP8)  # K % 128 != 0: no fp8 fallback
    B8 = _colmajor(torch.zeros(96, 256, device="cuda").to(FP8))
    assert gemm.kernel_for(A8, B8) == "unsupported"
    with pytest.raises(RuntimeError):
        gemm.matmul(A8, B8)


def test_fp8_bench_loop():
    A8, _ = gemm.fp8_quantize(torch.randn(8192, 8192, device="cuda"))
    B8, _ = gemm.fp8_quantize(torch.randn(8192, 8192, device="cuda"), colmajor=True)
    C = torch.empty(8192, 8192, device="cuda", dtype=torch.bfloat16)
    ms = gemm.bench_matmul(A8, B8, C, 10, 3) / 10
    tflops = 2 * 8192 ** 3 / ms / 1e9
    assert tflops > 1500, tflops  # above any bf16 rate: the fp8 MFMA path really runs


@pytest.mark.parametrize("M,N,batch", [(1024, 16384, 1), (16384, 1024, 1), (1024, 16384, 2)])
def test_fp8_thin_supertiles_exact(M, N, batch):
    """4 x 64 / 64 x 4-tile rounds (map_tile supertiles 4 / 5): every tile written once."""
    g = torch.Generator(device="cuda").manual_seed(M + N + batch)
    K = 256
    Af = torch.stack([_ints((M, K), g) for _ in range(batch)])
    Bf = torch.stack([_ints((K, N), g) for _ in range(batch)])
    A8 = Af.to(FP8)
    B8 = Bf.transpose(-1, -2).contiguous().to(FP8).transpose(-1, -2)
    if batch == 1:
        A8, B8, Af, Bf = A8[0], B8[0], Af[0], Bf[0]
    C = torch.full(torch.broadcast_shapes(Af.shape[:-1] + (N,)), float("nan"), device="cuda",
                   dtype=torch.bfloat16)
    gemm.matmul(A8, B8, out=C)
    assert torch.equal(C, (Af.double() @ Bf.double()).to(torch.bfloat16))


@pytest.mark.parametrize("batch,M,N,K", [(1, 256, 256, 768), (1, 1024, 2048, 1024), (1, 4096, 4096, 768),
                                         (1, 8192, 4096, 1024), (2, 2048, 2048, 768), (1, 16384, 2048, 768),
                                         (1, 2048, 16384, 768), (1, 8192, 8192, 512), (2, 4096, 2048, 512),
                                         (1, 16384, 2048, 512), (1, 256, 512, 512)])
def test_fp8_streaming_w4s_matches_w4_bitwise(batch, M, N, K):
    """fp8 W4S (one K-tile stream per CU, epilogue overlapped with the next
    tile's first DMAs, C = 0 MFMA starts): the same accumulation order as the
    W4 fp8 kernel, so bitwise equal, for one and several tiles per CU, uneven
    tile counts, thin grids and batches; K = 512 runs the K4 form (round 6)."""
    g = torch.Generator(device="cuda").manual_seed(batch + M + 3 * N + K)
    A = torch.randn(batch, M, K, device="cuda", generator=g).to(FP8)
    B = _colmajor(torch.randn(batch, K, N, device="cuda", generator=g).to(FP8))
    if batch == 1:
        A, B = A[0], B[0]
    ref = gemm.matmul(A, B, kernel="fp8_w4", alpha=0.5)
    for _ in range(2):
        out = torch.full_like(ref, float("nan"))
        gemm.matmul(A, B, out=out, kernel="fp8_w4s", alpha=0.5)
        assert torch.equal(out, ref)


@pytest.mark.parametrize("kernel", ["x_fp8_w4s_k4", "x_fp8_w4s_k4_tstore"])
@pytest.mark.parametrize("batch,M,N,K", [(1, 4096, 4096, 512), (1, 8192, 8192, 512), (2, 2048, 2048, 512),
                                         (1, 16384, 2048, 512), (1, 2048, 16384, 512), (1, 256, 256, 512),
                                         (1, 8192, 4096, 1024), (1, 4096, 4096, 768)])
def test_fp8_w4s_k4_matches_w4_bitwise(kernel, batch, M, N, K):
    """fp8 W4S down to four K-tiles (round 6, K4: the first pair's DMA targets
    through the same selects as the last pair's; at K = 512 the first pair
    already fetches the next tile's B(0)): bitwise equal to fp8 W4 with alpha,
    one and many tiles per CU, thin grids, batches, K = 512 / 768 / 1024."""
    g = torch.Generator(device="cuda").manual_seed(7 * batch + M + 3 * N + K)
    A = torch.randn(batch, M, K, device="cuda", generator=g).to(FP8)
    B = _colmajor(torch.randn(batch, K, N, device="cuda", generator=g).to(FP8))
    if batch == 1:
        A, B = A[0], B[0]
    ref = gemm.matmul(A, B, kernel="fp8_w4", alpha=0.5)
    for _ in range(2):
        out = torch.full_like(ref, float("nan"))
        gemm.matmul(A, B, out=out, kernel=kernel, alpha=0.5)
        assert torch.equal(out, ref)


def test_fp8_w4s_plan_and_refusals():
    g = torch.Generator(device="cuda").manual_seed(9)

    def ops(M, N, K):
        return (torch.randn(M, K, device="cuda", generator=g).to(FP8),
                _colmajor(torch.randn(K, N, device="cuda", generator=g).to(FP8)))

    A, B = ops(8192, 8192, 1024)  # 1024 tiles, K / 128 even: auto streams
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4s"
    with gemm.shared_device():
        assert gemm.kernel_for(A, B) == "pdmb_fp8_w4_nt"
    A, B = ops(8000, 8192, 1024)  # edge tiles: W4 fp8 only
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4_nt"
    with pytest.raises(RuntimeError):
        gemm.matmul(A, B, kernel="fp8_w4s")
    A, B = ops(8192, 8192, 640)  # K / 128 odd
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4_nt"
    with pytest.raises(RuntimeError):
        gemm.matmul(A, B, kernel="fp8_w4s")
    A, B = ops(8192, 8192, 512)  # four K-tiles (round 6): W4S's K4 form
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4s"
    A, B = ops(4096, 4096, 512)  # one tile per CU: W4
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4_nt"
    A, B = ops(8192, 8192, 256)  # two K-tiles: no stream
    assert gemm.kernel_for(A, B) == "pdmb_fp8_w4_nt"
    with pytest.raises(RuntimeError):
        gemm.matmul(A, B, kernel="fp8_w4s")


@pytest.mark.parametrize("M,N,K,splitk", [(8192, 1024, 8192, 0), (4096, 512, 4096, 0), (4096, 1024, 4096, 2),
                                          (2048, 2048, 2048, 4), (1000, 1052, 4096, 0)])
def test_fp8_splitk_exact(M, N, K, splitk):
    """fp8 W4 split-K (auto for grids that fill <= half the CUs, or forced):
    slices meet in-launch (splitk.h), alpha applied after the slot sum; exact
    on small integers, edge tiles included."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    Af, Bf = _ints((M, K), g, -2, 3), _ints((K, N), g, -2, 3)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    S = gemm.splitk_for(A8, B8, kernel="fp8_w4") if splitk == 0 else splitk
    if splitk == 0:
        assert S > 1, (M, N, K, S)  # these grids fill at most half the chip, >= 16 K-tiles / slice
    for _ in range(2):  # counters re-zeroed by every launch
        C = gemm.matmul(A8, B8, splitk=splitk, alpha=0.5, kernel="fp8_w4")
        assert torch.equal(C, (0.5 * (Af.double() @ Bf.double())).to(torch.bfloat16))


@pytest.mark.parametrize("M,N,K,S", [(768, 768, 8192, 3), (512, 512, 8192, 3), (1024, 768, 8192, 2),
                                     (1000, 260, 8192, None)])
def test_fp8_small_grid_split_plans_exact(M, N, K, S, monkeypatch):
    """Round 5 small-grid split rules (reducer-latency term, T128 x 3 below 32
    K-tiles per slice) on fp8 T128: the plan auto prices is the one launched;
    exact on small integers with masked edges; bitwise repeatable."""
    monkeypatch.delenv("PDMB_SPLIT_SLOT_LAT", raising=False)
    monkeypatch.delenv("PDMB_SPLIT3_SMALL", raising=False)
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    Af, Bf = _ints((M, K), g, -2, 3), _ints((K, N), g, -2, 3)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    if S is not None:
        assert gemm.kernel_for(A8, B8) == "pdmb_fp8_t128_nt"
        assert gemm.splitk_for(A8, B8) == S
    ref = (0.5 * (Af.double() @ Bf.double())).to(torch.bfloat16)
    C = gemm.matmul(A8, B8, alpha=0.5)
    assert torch.equal(C, ref)
    for _ in range(5):
        assert torch.equal(gemm.matmul(A8, B8, alpha=0.5), C)


# ---- fp8 tile family (gemm_tile.hip, DT = kFP8): under-filled fp8 grids ----
@pytest.mark.parametrize("kernel", ["fp8_t128", "fp8_t256x128", "fp8_t192", "fp8_t192x128"])
@pytest.mark.parametrize("M,N,K,splitk", [(256, 128, 128, 1), (512, 384, 256, 1), (2048, 2048, 2048, 1),
                                          (4096, 512, 4096, 0), (4096, 512, 4096, 2), (2048, 1024, 4096, 4),
                                          (1024, 16384, 256, 1), (16384, 1024, 256, 1), (768, 640, 1152, 2),
                                          (2048, 1024, 4096, 3)])
def test_fp8_tile_family_exact(kernel, M, N, K, splitk):
    """fp8 T128 / T256x128 (A / Bt images with the fp8 swizzle, one 16x16x128
    MFMA per block per K-tile, alpha in the LDS-staged epilogue) on exact small
    integers: unsplit, auto and forced split-K (odd K-tile counts too), and
    thin grids (map_tile supertiles 4 / 5 at 128-row tiles)."""
    if kernel == "fp8_t256x128" and M % 256:
        pytest.skip("T256x128: M % 256")
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + splitk)
    Af, Bf = _ints((M, K), g, -2, 3), _ints((K, N), g, -2, 3)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    assert gemm.kernel_for(A8, B8, kernel=kernel) == f"pdmb_{kernel}_nt"
    ref = (0.5 * (Af.double() @ Bf.double())).to(torch.bfloat16)
    for _ in range(2):  # split-K counters re-zeroed by every launch
        C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        gemm.matmul(A8, B8, out=C, kernel=kernel, splitk=splitk, alpha=0.5)
        assert torch.equal(C, ref)


@pytest.mark.parametrize("kernel", ["fp8_t128", "fp8_t256x128", "fp8_t192", "fp8_t192x128"])
def test_fp8_tile_family_matches_w4_bitwise(kernel):
    """Unsplit, a block's K-tiles go through the same one-MFMA-per-128-K chain
    as in fp8 W4: bitwise equal on random operands, batched too."""
    g = torch.Generator(device="cuda").manual_seed(21)
    A = torch.randn(2, 1024, 2048, device="cuda", generator=g).to(FP8)
    B = _colmajor(torch.randn(2, 2048, 768, device="cuda", generator=g).to(FP8))
    ref = gemm.matmul(A, B, kernel="fp8_w4", alpha=0.25, splitk=1)
    out = gemm.matmul(A, B, kernel=kernel, alpha=0.25, splitk=1)
    assert torch.equal(out, ref)


def test_fp8_tile_family_refusals_and_race_screen():
    g = torch.Generator(device="cuda").manual_seed(4)
    A = torch.randn(1000, 512, device="cuda", generator=g).to(FP8)
    B = _colmajor(torch.randn(512, 522, device="cuda", generator=g).to(FP8))  # N % 4 != 0
    assert gemm.kernel_for(A, B, kernel="fp8_t128") == "unsupported"
    A8, sa = gemm.fp8_quantize(torch.randn(4096, 4096, device="cuda", generator=g))
    B8, sb = gemm.fp8_quantize(torch.randn(4096, 512, device="cuda", generator=g), colmajor=True)
    ref = gemm.matmul(A8, B8, alpha=sa * sb, kernel="fp8_t128")
    assert _relerr(ref, (A8.double() * sa) @ (B8.double() * sb)) < 8e-3
    for _ in range(20):
        assert torch.equal(gemm.matmul(A8, B8, alpha=sa * sb, kernel="fp8_t128"), ref)


def test_fp8_planner_choices():
    """Auto on the reference's default sizes and their matrix_parallel shards
    (profiles/r2_fp8_tile_family_ab.jsonl): the fp8 tile family for grids
    that under-fill the 256 CUs with 256^2 tiles, W4 at one tile per CU,
    W4S from two."""
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("planner constants are for the 256-CU MI355X")

    def pick(M, N, K):
        A = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).to(FP8)
        B = _colmajor(torch.empty(K, N, device="cuda", dtype=torch.bfloat16).to(FP8))
        return gemm.kernel_for(A, B)

    assert pick(2048, 2048, 2048) == "pdmb_fp8_t128_nt"
    assert pick(4096, 512, 4096) == "pdmb_fp8_t128_nt"
    assert pick(4096, 1024, 4096) == "pdmb_fp8_t128_nt"
    assert pick(8192, 1024, 8192) == "pdmb_fp8_t256x128_nt"
    assert pick(4096, 4096, 4096) == "pdmb_fp8_w4_nt"
    assert pick(16384, 16384, 16384) == "pdmb_fp8_w4s"
    with gemm.shared_device():
        assert pick(16384, 16384, 16384) == "pdmb_fp8_w4_nt"


@pytest.mark.parametrize("kernel", ["fp8_t128", "fp8_t256x128"])
@pytest.mark.parametrize("M,N,K,splitk", [(300, 516, 256, 1), (1000, 1000, 512, 1), (700, 264, 2048, 2)])
def test_fp8_tile_family_edge_tiles(kernel, M, N, K, splitk):
    """fp8 tile family edge tiles: A and Bt rows past M / N load zeros through the
    descriptor extents; the bf16 stores are masked (N % 4)."""
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + K)
    Af, Bf = _ints((M, K), g, -2, 3), _ints((K, N), g, -2, 3)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=torch.bfloat16)
    out = big[:M, :N]
    assert gemm.kernel_for(A8, B8, out, kernel=kernel) == f"pdmb_{kernel}_nt"
    gemm.matmul(A8, B8, out=out, kernel=kernel, splitk=splitk, alpha=0.5)
    assert torch.equal(out, (0.5 * (Af.double() @ Bf.double())).to(torch.bfloat16))
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()


@pytest.mark.experiments
@pytest.mark.parametrize("M,N,K,form", [(6144, 6144, 6144, None), (6000, 6000, 6144, None),
                                        (7168, 7168, 1024, None), (7168, 7168, 7168, None),
                                        (6144, 6144, 6144, "rows"), (6000, 6000, 6144, "rows")])
def test_fp8_wave_tail_split(M, N, K, form, monkeypatch):  # forced forms: experiments build
    """fp8 wave-quantisation tail (gemm_dispatch.cpp tail_plan on fp8 W4): the
    whole waves as one fp8 W4 / W4S launch — whole tile rows, or (tile-range
    form) the first k x 256 tiles of the tile order — and the rest split-K in a
    second; exact on small integers (alpha folded in), nothing written outside
    C, the same bits every launch and under graph replay. form "rows": the
    tile-range form disabled (PDMB_TILE_TAIL=0), the row form runs."""
    if form == "rows":
        monkeypatch.setenv("PDMB_TILE_TAIL", "0")
    monkeypatch.setenv("PDMB_TAIL_REFINE", "0")  # the split-K forms (refined: test_gemm_gpu.py)
    monkeypatch.setenv("PDMB_T192", "0")  # else a whole 192-row tile plan beats the split forms
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    Af, Bf = _ints((M, K), g, -2, 3), _ints((K, N), g, -2, 3)
    A8, B8 = Af.to(FP8), _colmajor(Bf.to(FP8))
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=torch.bfloat16)
    out = big[:M, :N]
    m1, S, t1, _ = gemm.tail_split_for(A8, B8, out)
    if K >= 6144:
        assert (0 < m1 < M and m1 % 256 == 0) != (t1 > 0) and S in (2, 4, 8), (m1, S, t1)
    if form == "rows":
        assert t1 == 0
    elif K >= 6144:  # 24 x 24 / 28 x 28 tiles: no row count cuts a whole wave, tiles do
        assert t1 > 0 and t1 % 256 == 0, (m1, S, t1)
    gemm.matmul(A8, B8, out=out, alpha=0.5)
    ref = (0.5 * (Af.double() @ Bf.double())).to(torch.bfloat16)
    assert torch.equal(out, ref)
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    for _ in range(3):
        assert torch.equal(gemm.matmul(A8, B8, alpha=0.5), ref)
    C2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert gemm.bench_matmul(A8, B8, C2, 3, 1, graph=True) > 0
    assert torch.equal(C2, (Af.double() @ Bf.double()).to(torch.bfloat16))


SK_SHAPES = [(1, 5120, 5120, 5120), (1, 4608, 4608, 3072), (1, 6000, 5888, 3072),
             (1, 7168, 7168, 1024), (2, 2560, 2560, 5120), (1, 3072, 3072, 8192)]


@pytest.mark.experiments
# mode 2 on 7168^2 x 1024 is not generated: 16 tiles left after the whole
# waves, fewer K-tiles than workgroups per XCD
@pytest.mark.parametrize("shape,mode", [(s, m) for m in ("1", "2") for s in SK_SHAPES
                                        if not (m == "2" and s == (1, 7168, 7168, 1024))])
def test_fp8_stream_k(shape, mode, monkeypatch):
    """fp8 stream-K (gemm_fp8_sk, forced by PDMB_STREAMK=1): the whole waves
    before the last 1-2 as one launch (none below two waves), the rest as 256
    equal shares of K-tiles — tiles shared by 2 or 3 workgroups meet in K order
    (splitk.h sk_meet), edge tiles and a batch included. Exact on small
    integers with alpha, nothing written outside C, the same bits every launch
    and under graph replay."""
    monkeypatch.setenv("PDMB_STREAMK", mode)  # 2: only the last partial wave stream-K
    b, M, N, K = shape
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + b)
    Af = torch.randint(-2, 3, (b, M, K), device="cuda", generator=g).float()
    Bf = torch.randint(-2, 3, (b, K, N), device="cuda", generator=g).float()
    A8 = Af.to(FP8)
    B8 = Bf.transpose(-1, -2).contiguous().to(FP8).transpose(-1, -2)
    if b == 1:
        A8, B8, Af, Bf = A8[0], B8[0], Af[0], Bf[0]
    big = torch.full((b, M + 16, N + 24), float("nan"), device="cuda", dtype=torch.bfloat16)
    out = big[:, :M, :N] if b > 1 else big[0, :M, :N]
    m1, S, t1, r = gemm.tail_split_for(A8, B8, out)
    assert m1 == 0 and r == 0 and 2 <= S <= 8 and t1 % 256 == 0, (m1, S, t1, r)
    gemm.matmul(A8, B8, out=out, alpha=0.5)
    ref = (0.5 * torch.matmul(Af.double(), Bf.double())).to(torch.bfloat16)
    assert torch.equal(out, ref)
    assert torch.isnan(big[..., N:]).all() and torch.isnan(big[:, M:]).all()
    for _ in range(3):
        assert torch.equal(gemm.matmul(A8, B8, alpha=0.5), ref)
    C2 = torch.empty_like(ref)
    assert gemm.bench_matmul(A8, B8, C2, 3, 1, graph=True) > 0
    assert torch.equal(C2, torch.matmul(Af.double(), Bf.double()).to(torch.bfloat16))


@pytest.mark.parametrize("kernel,base", [("x_fp8_w4s_thin", "fp8_w4s"), ("x_w4s_thin", "w4s")])
@pytest.mark.parametrize("M,N,K", [(4096, 16384, 1024), (2048, 16384, 1024), (16384, 4096, 1024),
                                   (16384, 2048, 1024), (8192, 8192, 1024)])
def test_thin_round_w4s_matches_shipping_bitwise(kernel, base, M, N, K):
    """W4S with the thin 256-tile round that follows the grid's aspect (round 6
    experiments, common.h thin_supertile; profiles/r8zj_thin_round.md): only
    the tile order changes, so bitwise equal to the shipping W4S, every tile
    written (NaN-filled output), wide 4 x 64 / 8 x 32 and tall 64 x 4 / 32 x 8
    rounds and a square grid."""
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    if kernel.startswith("x_fp8"):
        A = torch.randn(M, K, device="cuda", generator=g).to(FP8)
        B = _colmajor(torch.randn(K, N, device="cuda", generator=g).to(FP8))
    else:
        A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        B = torch.randn(K, N, device="cuda", generator=g).to(torch.bfloat16)
    ref = gemm.matmul(A, B, kernel=base)
    out = torch.full_like(ref, float("nan"))
    gemm.matmul(A, B, out=out, kernel=kernel)
    assert torch.equal(out, ref)
