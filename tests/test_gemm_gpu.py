"""Numerics of the native gfx950 GEMM kernels against a plain PyTorch fp32/fp64
reference of the same op (cdna rule: A=I with asymmetric B, exact small-integer
data, full-tensor norm-relative error on random data)."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.ops import _native, gemm

pytestmark = pytest.mark.gpu

DT = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}
# norm-relative error budgets (output rounding dominates for 16-bit outputs)
TOL = {torch.bfloat16: 8e-3, torch.float16: 1.5e-3, torch.float32: 2e-6}


def _ref(A, B):
    return torch.matmul(A.double(), B.double())


def _relerr(C, R):
    return ((C.double() - R).norm() / R.norm().clamp_min(1e-30)).item()


def test_native_extension_is_loaded():
    mod = _native.load(build_if_missing=False)
    assert mod.ARCH == "gfx950"
    assert mod.__file__.endswith(".so")


# shipping LDS-DMA kernels + the 8-wave A/B schedules (those run only on a
# PDMB_EXPERIMENTS=1 build; the default build must refuse them)
FAST = ["mfma256d", "mfma256", "mfma256b", "mfma256c"]


TILED = ("pdmb_w4_nn", "pdmb_t256x128_nn", "pdmb_t128_nn", "pdmb_t128x2_nn", "pdmb_w4s",
         "pdmb_t192_nn", "pdmb_t192x128_nn")
F32 = ("pdmb_f32_256s_nn", "pdmb_f32_w4_nn", "pdmb_f32_t128_nn", "pdmb_f32_t128x2_nn", "pdmb_f32_t64_nn",
       "pdmb_f32_t64x2_nn", "pdmb_f32_w4l_nn")


def _need(kernel):
    """Skip an experiment-kernel case on the default (shipping) build."""
    if kernel in gemm.EXPERIMENT_KERNELS and not gemm.experiments_built():
        with pytest.raises(ValueError):
            gemm._kid(kernel)
        pytest.skip(f"{kernel} is an experiment kernel (PDMB_EXPERIMENTS=1 build)")


@pytest.mark.parametrize("kernel", FAST)
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 128), (1000, 1048, 320),
                                   (300, 200, 128), (4352, 4352, 448)])
def test_mfma256_exact_small_integers(dtype, M, N, K, kernel):
    _need(kernel)
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    A = torch.randint(-1, 2, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-1, 2, (K, N), device="cuda", generator=g).to(dt)
    assert gemm.kernel_for(A, B, kernel=kernel) == gemm.KERNEL_NAMES[gemm._kid(kernel)]
    C = gemm.matmul(A, B, kernel=kernel)
    R = _ref(A, B)  # |R| <= K <= 448: exact in fp16; bf16 rounds > 256 only
    if dt == torch.float16 or K <= 256:
        assert torch.equal(C.double(), R)
    else:
        assert _relerr(C, R) < TOL[dt]


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_mfma256_identity_asymmetric(dtype):
    dt = DT[dtype]
    n = 512
    A = torch.eye(n, device="cuda", dtype=dt)
    B = (torch.arange(n, device="cuda").view(n, 1) * 3 + torch.arange(n, device="cuda").view(1, n) * 0.5)
    B = (B % 61).to(dt)
    C = gemm.matmul(A, B)
    assert torch.equal(C, B)
    C2 = gemm.matmul(B, A)
    assert torch.equal(C2, B)


@pytest.mark.parametrize("kernel", FAST)
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("n", [2048, 4096])
def test_mfma256_random(dtype, n, kernel):
    _need(kernel)
    dt = DT[dtype]
    torch.manual_seed(0)
    A = torch.randn(n, n, device="cuda", dtype=dt)
    B = torch.randn(n, n, device="cuda", dtype=dt)
    C = gemm.matmul(A, B, kernel=kernel)
    R = torch.matmul(A.float(), B.float()).double()
    assert _relerr(C, R) < TOL[dt]


@pytest.mark.parametrize("kernel", FAST)
def test_mfma256_batched_and_broadcast(kernel):
    _need(kernel)
    dt = torch.bfloat16
    torch.manual_seed(1)
    A = torch.randn(3, 512, 320, device="cuda", dtype=dt)
    B = torch.randn(3, 320, 768, device="cuda", dtype=dt)
    B = torch.randn(3, 384, 768, device="cuda", dtype=dt)[:, :320]  # strided batch
    C = gemm.bmm(A, B, kernel=kernel)
    R = torch.bmm(A.double(), B.double())
    assert _relerr(C, R) < TOL[dt]
    B2 = torch.randn(320, 768, device="cuda", dtype=dt)
    C2 = gemm.matmul(A, B2, kernel=kernel)
    assert _relerr(C2, torch.matmul(A.double(), B2.double())) < TOL[dt]


def test_mfma256_column_shard_views():
    """matrix_parallel computes A @ B[:, shard] — a strided column view."""
    dt = torch.bfloat16
    torch.manual_seed(2)
    A = torch.randn(1024, 1024, device="cuda", dtype=dt)
    B = torch.randn(1024, 1024, device="cuda", dtype=dt)
    for ws in (2, 4, 8):
        cols = 1024 // ws
        for r in range(ws):
            Bs = B[:, r * cols:(r + 1) * cols]
            C = gemm.matmul(A, Bs)
            assert _relerr(C, _ref(A, Bs)) < TOL[dt]


def test_out_is_written_in_place_and_stream_ordered():
    dt = torch.bfloat16
    A = torch.randn(512, 512, device="cuda", dtype=dt)
    B = torch.randn(512, 512, device="cuda", dtype=dt)
    out = torch.full((512, 512), float("nan"), device="cuda", dtype=dt)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        r = gemm.matmul(A, B, out=out)
    s.synchronize()
    assert r.data_ptr() == out.data_ptr()
    assert not torch.isnan(out).any()


@pytest.mark.parametrize("dtype", ["bfloat16", "float16", "float32"])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (100, 72, 50), (257, 129, 33), (640, 384, 512),
                                   (129, 1000, 1001)])
def test_generic_random(dtype, M, N, K):
    dt = DT[dtype]
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", dtype=dt)
    B = torch.randn(K, N, device="cuda", dtype=dt)
    C = gemm.matmul(A, B, kernel="generic")
    assert _relerr(C, _ref(A, B)) < TOL[dt]
    # auto must also be right (it may pick either kernel)
    C2 = gemm.matmul(A, B)
    assert _relerr(C2, _ref(A, B)) < TOL[dt]


def test_generic_unaligned_strides():
    dt = torch.bfloat16
    A = torch.randn(300, 203, device="cuda", dtype=dt)[:, 1:202]  # lda=203, misaligned base
    B = torch.randn(201, 150, device="cuda", dtype=dt)
    assert gemm.kernel_for(A, B) == "pdmb_generic_nn"
    C = gemm.matmul(A, B)
    assert _relerr(C, _ref(A, B)) < TOL[dt]


def test_fp32_exact_mfma_path():
    torch.manual_seed(3)
    A = torch.randn(512, 512, device="cuda", dtype=torch.float32)
    B = torch.randn(512, 512, device="cuda", dtype=torch.float32)
    # 4 256-tiles: a smaller fp32 tile (128x128, or 64x128 since round 5)
    assert gemm.kernel_for(A, B) in ("pdmb_f32_t128_nn", "pdmb_f32_t64_nn", "pdmb_f32_t64x2_nn")
    for k in ("auto", "generic", "f32_256s", "f32_w4", "f32_t128", "f32_t64", "f32_t64x2"):
        C = gemm.matmul(A, B, kernel=k)
        assert _relerr(C, _ref(A, B)) < TOL[torch.float32]


def test_zero_k():
    A = torch.randn(64, 0, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(0, 64, device="cuda", dtype=torch.bfloat16)
    out = torch.ones(64, 64, device="cuda", dtype=torch.bfloat16)
    gemm.matmul(A, B, out=out)
    assert (out == 0).all()


@pytest.mark.parametrize("graph", [False, True])
def test_native_bench_loop(graph):
    A = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(1024, 1024, device="cuda", dtype=torch.bfloat16)
    ms = gemm.bench_matmul(A, B, out, iters=5, warmup=2, graph=graph)
    assert ms > 0
    assert _relerr(out, _ref(A, B)) < TOL[torch.bfloat16]


@pytest.mark.parametrize("kernel", FAST)
def test_race_screen_repeated_runs(kernel):
    """LDS-DMA pipeline race screen: identical outputs over many launches at several
    sizes, including one big enough to keep every CU busy for many rounds."""
    _need(kernel)
    for n in (768, 2048, 2560, 8192):
        torch.manual_seed(n)
        A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        ref = gemm.matmul(A, B, kernel=kernel)
        R = torch.matmul(A.float(), B.float()).double()
        assert _relerr(ref, R) < TOL[torch.bfloat16]
        for _ in range(10 if n == 8192 else 20):
            assert torch.equal(gemm.matmul(A, B, kernel=kernel), ref)


@pytest.mark.parametrize("M,N,K", [(256, 256, 32), (512, 768, 96), (1000, 1052, 320),
                                   (300, 200, 64), (2304, 2048, 1024)])
@pytest.mark.parametrize("kernel", ["f32_256", "f32_256s", "f32_w4", "x_f32_256s_direct", "f32_t128",
                                    "f32_t128x2", "x_f32_w4_b32", "x_f32_t128_b32", "f32_t64", "f32_t64x2",
                                    "f32_w4l"])
def test_f32_256_exact_and_random(M, N, K, kernel):
    _need(kernel)
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).float()
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).float()
    assert gemm.kernel_for(A, B, kernel=kernel).startswith(("pdmb_f32_256", "pdmb_f32_w4", "pdmb_f32_t128",
                                                            "pdmb_f32_t64"))
    C = gemm.matmul(A, B, kernel=kernel)
    assert torch.equal(C.double(), _ref(A, B))  # small integers: exact in fp32
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(K, N, device="cuda", generator=g)
    C = gemm.matmul(A, B, kernel=kernel)
    assert _relerr(C, _ref(A, B)) < TOL[torch.float32]


@pytest.mark.parametrize("kernel", ["f32_w4", "f32_t128", "f32_t64", "f32_t64x2"])
@pytest.mark.parametrize("M,N,K,splitk,split", [(4096, 1024, 4096, 0, None), (4096, 2048, 4096, 0, None),
                                                (2048, 2048, 2048, 0, None), (1000, 1052, 4096, 0, True),
                                                (512, 512, 1024, 2, True), (4096, 4096, 4096, 0, False),
                                                (1000, 1052, 4096, 4, True), (700, 300, 2048, 8, True),
                                                (1000, 1052, 4096, 3, True), (1000, 300, 8192, 5, True),
                                                (700, 300, 8192, 6, True)])
def test_f32_splitk_exact(kernel, M, N, K, splitk, split):
    """Exact-fp32 W4 / T128 split-K for under-filled grids (matrix_parallel's
    fp32 shards): slices meet in-launch (splitk.h), edge tiles masked; exact on
    small integers, and bitwise stable across launches (slot sums in slice
    order). ``split``: whether the planner must split (None: either)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).float()
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).float()
    assert gemm.kernel_for(A, B, kernel=kernel) == f"pdmb_{kernel}_nn"
    assert gemm.kernel_for(A, B) in F32
    S = gemm.splitk_for(A, B, kernel=kernel, splitk=splitk)
    if splitk:
        assert S == splitk
    elif split is not None:
        assert (S > 1) == split, S
    ref = _ref(A, B)
    for _ in range(2):  # counters re-zeroed by every launch
        big = torch.full((M + 8, N + 12), float("nan"), device="cuda")
        C = big[:M, :N]
        gemm.matmul(A, B, out=C, kernel=kernel, splitk=splitk)
        assert torch.equal(C.double(), ref)
        assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(K, N, device="cuda", generator=g)
    C = gemm.matmul(A, B, kernel=kernel, splitk=splitk)
    assert _relerr(C, _ref(A, B)) < TOL[torch.float32]
    assert torch.equal(gemm.matmul(A, B, kernel=kernel, splitk=splitk), C)


@pytest.mark.parametrize("M,N,K,kernel,S", [(2560, 2048, 4096, "f32_t64x2", 2), (1024, 256, 16384, "f32_t64", 8),
                                             (512, 12288, 2048, "f32_t128x2", 2), (1000, 3000, 4096, None, None),
                                             (1536, 3072, 1024, "f32_t64x2", 2), (1536, 1536, 4096, "f32_t64x2", 4),
                                             (3584, 3584, 2048, "f32_t64x2", 2), (4608, 4608, 4096, "f32_t64x2", 2)])
def test_f32_auto_x2_split_and_split8_exact(M, N, K, kernel, S, monkeypatch):
    """Round 5 planner: auto runs f32_t128x2 split >= 3 slices per CU on grids
    of < 2 tiles per CU, f32_t64x2 split there, and 8-way fp32 splits
    (test_planner_cpu.py). The plan
    auto prices is the one that launches; exact on small integers (edges
    masked), bitwise repeatable on random data."""
    monkeypatch.delenv("PDMB_F32X2SPLIT", raising=False)
    monkeypatch.delenv("PDMB_SPLIT8", raising=False)
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).float()
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).float()
    if kernel:
        assert gemm.kernel_for(A, B) == f"pdmb_{kernel}_nn"
        assert gemm.splitk_for(A, B) == S
    big = torch.full((M + 8, N + 12), float("nan"), device="cuda")
    gemm.matmul(A, B, out=big[:M, :N])
    assert torch.equal(big[:M, :N].double(), _ref(A, B))
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(K, N, device="cuda", generator=g)
    C = gemm.matmul(A, B)
    assert _relerr(C, _ref(A, B)) < TOL[torch.float32]
    for _ in range(5):
        assert torch.equal(gemm.matmul(A, B), C)


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("M,N,K,S", [(768, 768, 4096, 3), (1024, 1024, 8192, 3), (256, 768, 2048, 3),
                                     (700, 304, 4096, 3)])
def test_small_grid_split_plans_exact(dtype, M, N, K, S, monkeypatch):
    """Round 5 small-grid split rules (reducer-latency term, T128 x 3 below 32
    K-tiles per slice; test_planner_cpu.py): the plan auto prices is the one
    launched; exact on small integers with masked edges; bitwise repeatable."""
    monkeypatch.delenv("PDMB_SPLIT_SLOT_LAT", raising=False)
    monkeypatch.delenv("PDMB_SPLIT3_SMALL", raising=False)
    dt = getattr(torch, dtype)
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(dt)
    if S is not None:
        assert gemm.kernel_for(A, B) == "pdmb_t128_nn"
        assert gemm.splitk_for(A, B) == S
    big = torch.full((M + 8, N + 12), float("nan"), device="cuda", dtype=dt)
    gemm.matmul(A, B, out=big[:M, :N])
    assert torch.equal(big[:M, :N], (A.double() @ B.double()).to(dt))
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = torch.randn(K, N, device="cuda", generator=g).to(dt)
    C = gemm.matmul(A, B)
    assert _relerr(C, _ref(A, B)) < TOL[dt]
    for _ in range(5):
        assert torch.equal(gemm.matmul(A, B), C)


F32_T128_ARMS = ["f32_t128", "f32_t128x2", "x_f32_t128_b32", "f32_t64", "f32_t64x2", "x_f32_t128_lean",
                 "x_f32_t128x2_lean", "x_f32_t64_lean", "x_f32_t64x2_lean"]


@pytest.mark.parametrize("M,N,K,b", [(128, 128, 32, 1), (256, 384, 96, 1), (1000, 1052, 320, 1),
                                     (300, 200, 64, 1), (384, 640, 256, 3), (4096, 512, 4096, 1),
                                     (1, 4, 32, 1), (129, 132, 1024, 2)])
@pytest.mark.parametrize("kernel", F32_T128_ARMS)
def test_f32_t128_exact_identity_and_batched(M, N, K, b, kernel):
    """The 128x128 exact-fp32 tile (gemm_f32_tile.hip; shipping: b128 B reads
    with column-permuted MFMAs; experiment arms: b32 B reads, 2 stages x 2
    workgroups per CU) and its 64x128 form (f32_t64): small integers exact (every fp32 partial sum exact),
    A = I with an asymmetric B (catches a column permutation the epilogue
    fails to undo), batched, edge tiles in M and N, one-K-tile problems."""
    _need(kernel)
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + b)
    A = torch.randint(-3, 4, (b, M, K), device="cuda", generator=g).float()
    B = torch.randint(-3, 4, (b, K, N), device="cuda", generator=g).float()
    if b == 1:
        A, B = A[0], B[0]
    C = gemm.matmul(A, B, kernel=kernel)
    assert torch.equal(C.double(), torch.matmul(A.double(), B.double()))
    n = 512
    I = torch.eye(n, device="cuda")
    Bs = (torch.arange(n * 640, device="cuda").view(n, 640) % 97).float()
    assert torch.equal(gemm.matmul(I, Bs, kernel=kernel), Bs)


@pytest.mark.parametrize("kernel", F32_T128_ARMS)
def test_f32_t128_race_screen(kernel):
    _need(kernel)
    torch.manual_seed(21)
    A = torch.randn(4096, 2048, device="cuda")
    B = torch.randn(2048, 1024, device="cuda")
    for S in (1, 2):
        ref = gemm.matmul(A, B, kernel=kernel, splitk=S)
        assert _relerr(ref, _ref(A, B)) < TOL[torch.float32]
        for _ in range(10):
            assert torch.equal(gemm.matmul(A, B, kernel=kernel, splitk=S), ref)


def test_f32_256_identity_batched_and_shards():
    n = 512
    A = torch.eye(n, device="cuda")
    B = (torch.arange(n * n, device="cuda").view(n, n) % 97).float()
    assert torch.equal(gemm.matmul(A, B), B) and torch.equal(gemm.matmul(B, A), B)
    torch.manual_seed(7)
    A3 = torch.randn(3, 384, 256, device="cuda")
    B3 = torch.randn(3, 256, 640, device="cuda")
    assert gemm.kernel_for(A3, B3) in F32  # 18 256-tiles of 8 K-tiles
    assert _relerr(gemm.bmm(A3, B3), torch.bmm(A3.double(), B3.double())) < TOL[torch.float32]
    Bf = torch.randn(1024, 1024, device="cuda")
    Af = torch.randn(1024, 1024, device="cuda")
    for r in range(4):  # matrix_parallel column shards (strided views)
        Bs = Bf[:, r * 256:(r + 1) * 256]
        assert _relerr(gemm.matmul(Af, Bs), _ref(Af, Bs)) < TOL[torch.float32]


@pytest.mark.experiments
@pytest.mark.parametrize("b,M,N,K,exact", [(1, 256, 256, 128, True), (1, 4096, 4096, 256, True),
                                           (1, 8192, 8192, 512, False), (1, 5120, 3072, 1024, True),
                                           (1, 9216, 6912, 640, True), (3, 1024, 1024, 512, True),
                                           (1, 2304, 8960, 384, False), (1, 4352, 4608, 192, True)])
def test_f32_w4s_exact_and_bitwise(b, M, N, K, exact):
    """The streamed exact-fp32 kernel (x_f32_w4s, round 6, experiments build:
    its first launches hung in 3 of 4 processes, gemm_f32_w4.hip): one K-tile stream per
    CU over static tiles (1 to 10 tiles per workgroup, grids that are not whole
    waves, a batch, the four-K-tile minimum). Small integers exact against
    fp64 (a dropped, doubled or misplaced K-tile of the stream would show), and
    bitwise equal to the unstreamed f32_w4 (the same per-element MFMA order)."""
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + b)
    sa, sb = ((b, M, K), (b, K, N)) if b > 1 else ((M, K), (K, N))
    if exact:
        A = torch.randint(-3, 4, sa, device="cuda", generator=g).float()
        B = torch.randint(-3, 4, sb, device="cuda", generator=g).float()
    else:
        A = torch.randn(sa, device="cuda", generator=g)
        B = torch.randn(sb, device="cuda", generator=g)
    _need("x_f32_w4s")
    assert gemm.kernel_for(A, B, kernel="x_f32_w4s") == "pdmb_f32_w4s"
    C = gemm.matmul(A, B, kernel="x_f32_w4s")
    R = torch.matmul(A.double(), B.double())
    if exact:
        assert torch.equal(C.double(), R)
    else:
        assert _relerr(C, R) < TOL[torch.float32]
    assert torch.equal(C, gemm.matmul(A, B, kernel="f32_w4"))


@pytest.mark.parametrize("b,M,N,K", [(1, 4096, 4096, 4096), (1, 8192, 2048, 8192), (1, 4096, 4096, 4128),
                                     (4, 2048, 2048, 4096), (1, 8192, 8192, 8192), (2, 4096, 4096, 4096)])
def test_f32_w4l_one_wave_auto_exact_and_bitwise(b, M, N, K):
    """Round 6: whole waves of 256x256 fp32 tiles (K >= 4096) run the lean W4
    K-loop (f32_w4l); small integers exact against fp64 (K / 32 odd at 4128:
    the branch-free loop's re-read tail), bitwise equal to f32_w4 (the same
    per-element MFMA order), A = I with an asymmetric B, and repeatable."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + b)
    sa, sb = ((b, M, K), (b, K, N)) if b > 1 else ((M, K), (K, N))
    A = torch.randint(-3, 4, sa, device="cuda", generator=g).float()
    B = torch.randint(-3, 4, sb, device="cuda", generator=g).float()
    assert gemm.kernel_for(A, B) == "pdmb_f32_w4l_nn"
    C = gemm.matmul(A, B)
    assert torch.equal(C.double(), torch.matmul(A.double(), B.double()))
    assert torch.equal(C, gemm.matmul(A, B, kernel="f32_w4"))
    for _ in range(3):
        assert torch.equal(gemm.matmul(A, B), C)
    if b == 1 and M == N == K:
        eye = torch.eye(M, device="cuda")
        Bq = (torch.arange(M * M, device="cuda").view(M, M) % 97).float()
        assert torch.equal(gemm.matmul(eye, Bq), Bq) and torch.equal(gemm.matmul(Bq, eye), Bq)
    with pytest.raises(RuntimeError):
        gemm.matmul(A, B, kernel="f32_w4l", splitk=2)  # unsplit only


@pytest.mark.parametrize("kernel", ["f32_256", "f32_256s", "f32_w4", "f32_t128", "f32_w4l"])
def test_f32_256_race_screen(kernel):
    _need(kernel)
    torch.manual_seed(11)
    A = torch.randn(4096, 4096, device="cuda")
    B = torch.randn(4096, 4096, device="cuda")
    ref = gemm.matmul(A, B, kernel=kernel)
    R = torch.matmul(A.double(), B.double())
    assert _relerr(ref, R) < TOL[torch.float32]
    for _ in range(10):
        assert torch.equal(gemm.matmul(A, B, kernel=kernel), ref)


@pytest.mark.parametrize("dtype", ["bfloat16", "float16", "float32"])
@pytest.mark.parametrize("M,N,K", [(2000, 1999, 1000), (1536, 1030, 2050)])
def test_odd_sizes_padded_to_fast_path(dtype, M, N, K):
    """Big problems with K / N off the fast kernels' granule run padded on the fast path."""
    dt = DT[dtype]
    torch.manual_seed(M + N)
    A = torch.randn(M, K, device="cuda", dtype=dt)
    B = torch.randn(K, N, device="cuda", dtype=dt)
    assert gemm.kernel_for(A, B) == "pdmb_generic_nn"  # unpadded, only generic could run it
    assert gemm.padded_kernel_for(A, B) in ("pdmb_mfma256d_nn",) + F32 + TILED
    C = gemm.matmul(A, B)
    assert C.shape == (M, N)
    assert _relerr(C, _ref(A, B)) < TOL[dt]
    out = torch.full((M, N), float("nan"), device="cuda", dtype=dt)
    assert gemm.matmul(A, B, out=out).data_ptr() == out.data_ptr()
    assert _relerr(out, _ref(A, B)) < TOL[dt]


def test_padded_path_misaligned_views_and_batches():
    torch.manual_seed(9)
    big = torch.randn(1100, 2051, device="cuda", dtype=torch.bfloat16)
    A = big[:, 1:2049]            # lda = 2051 (misaligned), K = 2048
    B = torch.randn(2048, 1500, device="cuda", dtype=torch.bfloat16)
    assert gemm.padded_kernel_for(A, B) in TILED  # M = 1100: masked edge tiles
    assert _relerr(gemm.matmul(A, B), _ref(A, B)) < TOL[torch.bfloat16]
    A3 = torch.randn(3, 700, 1000, device="cuda", dtype=torch.float16)
    B3 = torch.randn(3, 1000, 1300, device="cuda", dtype=torch.float16)
    assert gemm.padded_kernel_for(A3, B3) in TILED
    assert _relerr(gemm.bmm(A3, B3), torch.bmm(A3.double(), B3.double())) < TOL[torch.float16]
    out = torch.empty(1100, 1500, device="cuda", dtype=torch.bfloat16)
    ms = gemm.bench_matmul(A, B, out, iters=3, warmup=1)  # native loop takes the padded path too
    assert ms > 0 and _relerr(out, _ref(A, B)) < TOL[torch.bfloat16]


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_padded_k_only_writes_c_in_place(dtype):
    """Only K off its granule: A / B are padded copies but the kernel writes the
    caller's C directly (no padded C, no unpad copy) — and nothing past N or M."""
    dt = DT[dtype]
    torch.manual_seed(13)
    A = torch.randn(1500, 1000, device="cuda", dtype=dt)
    B = torch.randn(1000, 1024, device="cuda", dtype=dt)
    assert gemm.kernel_for(A, B) == "pdmb_generic_nn" and gemm.padded_kernel_for(A, B) is not None
    big = torch.full((1504, 1048), float("nan"), device="cuda", dtype=dt)
    out = big[:1500, :1024]
    gemm.matmul(A, B, out=out)
    assert _relerr(out, _ref(A, B)) < TOL[dt]
    assert torch.isnan(big[:, 1024:]).all() and torch.isnan(big[1500:]).all()


# ---- W4: 4 waves x 128x128 per wave (gemm_w4.hip), the auto kernel for whole 256-tiles ----

@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("b,M,N,K,pad", [(1, 256, 256, 64, 0), (1, 1024, 512, 192, 0),
                                         (3, 512, 768, 256, 0), (1, 768, 1280, 320, 64),
                                         (1, 2304, 2048, 1024, 0)])
def test_w4_exact_small_integers(dtype, b, M, N, K, pad):
    """Integer operands keep every fp32 partial sum exact: C == fp64 product rounded once."""
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    A = torch.randint(-3, 4, (b, M, K + pad), device="cuda", generator=g).to(dt)[..., :K]
    B = torch.randint(-3, 4, (b, K, N + pad), device="cuda", generator=g).to(dt)[..., :N]
    if b == 1:
        A, B = A[0], B[0]
    # auto picks a whole-tile kernel (W4, or a smaller tile for these under-filled grids)
    assert gemm.kernel_for(A, B) in TILED
    C = gemm.matmul(A, B, kernel="w4")
    assert torch.equal(C, (A.double() @ B.double()).to(dt))


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_w4_random_matches_sched3(dtype):
    dt = DT[dtype]
    torch.manual_seed(5)
    A = torch.randn(4096, 4096, device="cuda", dtype=dt)
    B = torch.randn(4096, 4096, device="cuda", dtype=dt)
    C = gemm.matmul(A, B, kernel="w4")
    assert _relerr(C, _ref(A, B)) < TOL[dt]
    # same fp32 accumulation order per output as the 8-wave kernel: bitwise equal
    assert torch.equal(C, gemm.matmul(A, B, kernel="mfma256d"))


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("b,M,N,K,splitk", [(1, 300, 512, 256, 0), (1, 1000, 1000, 512, 0),
                                           (1, 257, 264, 128, 0), (2, 700, 1304, 1024, 0),
                                           (1, 16000, 16000, 128, 0), (1, 3000, 520, 4096, 2)])
def test_w4_edge_tiles_masked(dtype, b, M, N, K, splitk):
    """M / N not multiples of 256 (N % 8 == 0): rows past M load zeros through
    the descriptor extent, B columns past N only feed dropped outputs, and the
    epilogue masks its stores — exact on small integers, unsplit and split, and
    nothing is written past N inside a wider row (ldc > N) or past M."""
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + b)
    A = torch.randint(-3, 4, (b, M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (b, K, N), device="cuda", generator=g).to(dt)
    big = torch.full((b, M + 16, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:, :M, :N]
    if b == 1:
        A, B, out = A[0], B[0], out[0]
    assert gemm.kernel_for(A, B, out, kernel="w4") == "pdmb_w4_nn"
    gemm.matmul(A, B, out=out, kernel="w4", splitk=splitk)
    assert torch.equal(out, (A.double() @ B.double()).to(dt))
    assert torch.isnan(big[..., :M, N:]).all() and torch.isnan(big[..., M:, :]).all()


@pytest.mark.parametrize("kernel", ["t128", "t256x128", "t128x2", "t192", "t192x128"])
@pytest.mark.parametrize("M,N,K,splitk", [(300, 520, 256, 1), (1000, 1000, 512, 1), (3000, 7000, 512, 1),
                                         (700, 264, 2048, 2), (700, 264, 2048, 3)])
def test_tile_family_edge_tiles_masked(kernel, M, N, K, splitk):
    """The tile family's edge tiles (M % BM, N % 128): exact small integers, and
    nothing written past N in a wider row or past M."""
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(M + 5 * N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(dt)
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:M, :N]
    assert gemm.kernel_for(A, B, out, kernel=kernel) == f"pdmb_{kernel}_nn"
    gemm.matmul(A, B, out=out, kernel=kernel, splitk=splitk)
    assert torch.equal(out, (A.double() @ B.double()).to(dt))
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()


# Forced tail forms (PDMB_TILE_TAIL / PDMB_TAIL_REFINE / PDMB_T192): the
# planner reads those A/B switches only in a PDMB_EXPERIMENTS=1 build, so these
# run there; test_shipping_tail_plans_exact covers the tails the shipping
# planner chooses by itself.
@pytest.mark.experiments
@pytest.mark.parametrize("M,N,K,form", [(6000, 6000, 6144, "tiles"), (10000, 10000, 10048, "tiles"),
                                        (6144, 6144, 6144, "tiles"), (7168, 7168, 7168, "tiles"),
                                        (6000, 6000, 6144, "rows"), (10000, 10000, 10048, "rows"),
                                        (6144, 6144, 6144, "rows")])
def test_auto_wave_tail_split(M, N, K, form, monkeypatch):
    """Auto's wave-quantisation tail: the whole waves as one W4 / W4S launch —
    the first k x 256 tiles of the tile order ("tiles", the default form) or
    whole tile rows ("rows": PDMB_TILE_TAIL=0) — and the rest split-K in a
    second. Exact small integers, nothing written past N in a wider row or
    past M, the same bits under graph replay."""
    if form == "rows":
        monkeypatch.setenv("PDMB_TILE_TAIL", "0")
    monkeypatch.setenv("PDMB_T192", "0")  # else a whole 192-row tile plan beats the split forms
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(dt)
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:M, :N]
    if form == "tiles":  # the split-K tile-range form (the refined one is tested below)
        monkeypatch.setenv("PDMB_TAIL_REFINE", "0")
    m1, S, t1, r = gemm.tail_split_for(A, B, out)
    if form == "rows":
        assert 0 < m1 < M and m1 % 256 == 0 and S in (2, 4) and t1 == 0 and r == 1, (m1, S, t1, r)
    else:
        assert m1 == 0 and t1 > 0 and t1 % 256 == 0 and S in (2, 4, 8) and r == 1, (m1, S, t1, r)
    gemm.matmul(A, B, out=out)
    ref = (A.double() @ B.double()).to(dt)
    assert torch.equal(out, ref)
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    C2 = torch.empty(M, N, device="cuda", dtype=dt)
    assert gemm.bench_matmul(A, B, C2, 3, 1, graph=True) > 0
    assert torch.equal(C2, ref)


@pytest.mark.parametrize("dtype", ["bfloat16", "float8_e4m3fn"])
def test_batched_tile_range_tail(dtype):
    """The tile-range tail over a batch (5120^3 x 2: 800 tiles = 768 in whole
    waves + 32 split-K; the tile order runs across batch elements): exact on
    small integers for every element, nothing written outside C."""
    dt = getattr(torch, dtype)
    fp8 = dt == gemm.FP8
    M = N = K = 5120
    g = torch.Generator(device="cuda").manual_seed(77)
    lo, hi = (-2, 3) if fp8 else (-3, 4)
    Af = torch.randint(lo, hi, (2, M, K), device="cuda", generator=g).float()
    Bf = torch.randint(lo, hi, (2, K, N), device="cuda", generator=g).float()
    if fp8:
        A, B = Af.to(dt), Bf.transpose(-1, -2).contiguous().to(dt).transpose(-1, -2)
    else:
        A, B = Af.to(dt), Bf.to(dt)
    odt = gemm.out_dtype(dt)
    big = torch.full((2, M + 8, N + 16), float("nan"), device="cuda", dtype=odt)
    out = big[:, :M, :N]
    m1, S, t1, r = gemm.tail_split_for(A, B, out)
    assert m1 == 0 and t1 == 768 and (S > 1 or r > 1), (m1, S, t1, r)
    gemm.matmul(A, B, out=out)
    ref = torch.matmul(Af.double(), Bf.double()).to(odt)
    assert torch.equal(out, ref)
    assert torch.isnan(big[:, :, N:]).all() and torch.isnan(big[:, M:]).all()


REFINED_SHAPES = [(6144, 6144, 6144, 2), (6000, 6000, 6144, 2), (4608, 4608, 3072, 2),
                  (6000, 5888, 3072, 4), (6144, 6144, 3072, 4), (4608, 4608, 3072, 4),
                  (6144, 4096, 4096, 2), (3000, 7000, 5056, 2)]


@pytest.mark.experiments  # PDMB_TAIL_REFINE=R forces the form (experiments build)
@pytest.mark.parametrize("dtype,M,N,K,R", [(d,) + s for d in ("bfloat16", "float16", "float8_e4m3fn")
                                           for s in REFINED_SHAPES
                                           if not (d == "float8_e4m3fn" and s[2] % 128)])  # fp8: K % 128
def test_refined_wave_tail(dtype, M, N, K, R, monkeypatch):
    """The refined tail (PDMB_TAIL_REFINE=R forces it): whole waves of 256x256
    tiles as one launch, the remaining tiles of the same order cut into R
    256x128 / 128x128 tiles of the tile family, unsplit — edge tiles (6000,
    5888; 3000 x 7000) included, and grids whose single launch would be the
    tile family itself (bf16 6144 x 4096 x 4096, 4608^2 x 3072): exact on small integers, nothing written outside C,
    the same bits under graph replay."""
    monkeypatch.setenv("PDMB_TAIL_REFINE", str(R))
    dt = getattr(torch, dtype)
    fp8 = dt == gemm.FP8
    g = torch.Generator(device="cuda").manual_seed(M + N + K + R)
    lo, hi = (-2, 3) if fp8 else (-3, 4)
    Af = torch.randint(lo, hi, (M, K), device="cuda", generator=g).float()
    Bf = torch.randint(lo, hi, (K, N), device="cuda", generator=g).float()
    A = Af.to(dt)
    B = Bf.t().contiguous().to(dt).t() if fp8 else Bf.to(dt)
    odt = gemm.out_dtype(dt)
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=odt)
    out = big[:M, :N]
    m1, S, t1, r = gemm.tail_split_for(A, B, out)
    assert m1 == 0 and S == 1 and t1 > 0 and t1 % 256 == 0 and r == R, (m1, S, t1, r)
    gemm.matmul(A, B, out=out)
    ref = (Af.double() @ Bf.double()).to(odt)
    assert torch.equal(out, ref)
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    C2 = torch.empty(M, N, device="cuda", dtype=odt)
    assert gemm.bench_matmul(A, B, C2, 3, 1, graph=True) > 0
    assert torch.equal(C2, ref)


@pytest.mark.parametrize("M,N,K", [(3072, 3072, 3072), (5120, 5120, 2048), (5120, 5120, 5120),
                                   (7168, 7168, 1024)])
def test_f32_wave_tail_split(M, N, K):
    """Exact fp32 tail (gemm_dispatch.cpp f32_tail_plan): the whole two-per-CU
    waves of 128x128 tiles as one f32_t128x2 launch (tile_end), the remaining
    tiles split S ways as one wave of f32_t128 (tile_span, meeting in-launch): exact on small integers, nothing written outside C, the same
    bits under graph replay."""
    dt = torch.float32
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(dt)
    m1, S, t1, r = gemm.tail_split_for(A, B)
    assert m1 == 0 and t1 > 0 and t1 % 512 == 0 and S > 1 and r == 1, (m1, S, t1, r)
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:M, :N]
    gemm.matmul(A, B, out=out)
    ref = (A.double() @ B.double()).to(dt)
    assert torch.equal(out, ref)
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()
    C2 = torch.empty(M, N, device="cuda", dtype=dt)
    assert gemm.bench_matmul(A, B, C2, 3, 1, graph=True) > 0
    assert torch.equal(C2, ref)


@pytest.mark.parametrize("M,N,K", [(6000, 6000, 6100), (6000, 5996, 6144)])
def test_padded_wave_tail_split(M, N, K):
    """The padded fast path (K or N off the granule) runs the padded problem with
    the same tail plan (6000 x 6000 x 6144 after padding): exact, nothing written
    outside C."""
    dt = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    A = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(dt)
    big = torch.full((M + 16, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:M, :N]
    assert gemm.padded_kernel_for(A, B) in TILED
    gemm.matmul(A, B, out=out)
    assert torch.equal(out, (A.double() @ B.double()).to(dt))
    assert torch.isnan(big[:, N:]).all() and torch.isnan(big[M:]).all()


def test_no_tail_split_where_it_does_not_pay():
    def tail(M, N, K, **kw):
        A = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.empty(K, N, device="cuda", dtype=torch.bfloat16)
        return gemm.tail_split_for(A, B, **kw)
    assert tail(16384, 16384, 16384) == (0, 1, 0, 1)   # whole waves
    assert tail(8192, 1024, 8192) == (0, 1, 0, 1)      # under-filled: the planner's split / small tiles
    assert tail(6000, 6000, 6144, kernel="w4") == (0, 1, 0, 1)  # explicit kernels run as asked


def test_w4_rejects_unaligned_n():
    A = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(256, 300, device="cuda", dtype=torch.bfloat16)  # N % 8 != 0
    assert gemm.kernel_for(A, B, kernel="w4") == "unsupported"
    with pytest.raises(RuntimeError):
        gemm.matmul(A, B, kernel="w4")


# ---- thin grids: 8x32 / 32x8-tile super-tile rounds (map_tile supertile 2 / 3) ----

@pytest.mark.parametrize("M,N,batch", [(2048, 8192, 1), (8192, 2048, 1), (2048, 8192, 2),
                                       (8192, 2048, 3), (4096, 2048, 1),
                                       (1024, 16384, 1), (16384, 1024, 1), (1024, 16384, 2)])
@pytest.mark.parametrize("kernel,dtype", [("w4", "bfloat16"), ("w4", "float16"),
                                          ("mfma256d", "bfloat16"), ("f32_256s", "float32"),
                                          ("f32_w4", "float32"), ("f32_t128", "float32")])
def test_thin_grid_supertiles_exact(M, N, batch, kernel, dtype):
    """Every output tile is written exactly once under the thin-grid block->tile
    maps (a mis-mapping leaves stale tiles or duplicates): integer data, exact
    result. Shapes: row chunks of an overlap GEMM, ws=8 column shards; 1024 x 16384
    and 16384 x 1024 are the 4 x 64 / 64 x 4-tile rounds (supertiles 4 / 5)."""
    dt, K = DT[dtype], 256
    g = torch.Generator(device="cuda").manual_seed(M + N + batch)
    A = torch.randint(-3, 4, (batch, M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (batch, K, N), device="cuda", generator=g).to(dt)
    if batch == 1:
        A, B = A[0], B[0]
    C = torch.full(torch.broadcast_shapes(A.shape[:-1] + (N,)), float("nan"), device="cuda",
                   dtype=dt)
    gemm.matmul(A, B, out=C, kernel=kernel)
    assert torch.equal(C, (A.double() @ B.double()).to(dt))


# ---- under-filled grids: T128 (128x128 tiles) and W4 / T128 split-K ----
# (matrix_parallel column shards at ws >= 4: 4096 x 512, 8192 x 1024; 2048^3)

WHOLE_TILE_SHAPES = [
    (2048, 2048, 2048, 1, 0), (4096, 512, 4096, 1, 0), (8192, 1024, 8192, 1, 2),
    (1024, 1024, 4096, 1, 2), (1024, 1024, 4096, 1, 4), (1024, 1024, 4096, 1, 8),
    (512, 512, 2048, 2, 4), (1024, 768, 832, 1, 4), (4096, 512, 4096, 1, 1),
    (256, 256, 64, 1, 0), (512, 768, 320, 3, 0)]


def _whole_tile_fits(kernel, M, N):
    """W4 needs M, N % 256; T256x128 needs M % 256 (the other combinations are
    not generated, rather than skipped)."""
    return not ((kernel == "w4" and (M % 256 or N % 256)) or (kernel == "t256x128" and M % 256))


@pytest.mark.parametrize("kernel,M,N,K,b,splitk", [
    (k,) + s for k in ("w4", "t256x128", "t128", "t128x2") for s in WHOLE_TILE_SHAPES
    if _whole_tile_fits(k, s[0], s[1])])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_whole_tile_kernels_exact(kernel, M, N, K, b, splitk, dtype):
    """Integer data keeps every fp32 slice partial and their sum exact: the
    (split) result equals the fp64 product rounded once (K = 832 leaves the
    last of 4 slices one K-tile; K = 64 is a one-K-tile prologue/tail)."""
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    A = torch.randint(-3, 4, (b, M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (b, K, N), device="cuda", generator=g).to(dt)
    if b == 1:
        A, B = A[0], B[0]
    assert gemm.kernel_for(A, B, kernel=kernel) == f"pdmb_{kernel}_nn"
    S = gemm.splitk_for(A, B, kernel=kernel, splitk=splitk)
    assert S == splitk if splitk else S >= 1
    C = torch.full(torch.broadcast_shapes(A.shape[:-1] + (N,)), float("nan"), device="cuda",
                   dtype=dt)
    gemm.matmul(A, B, out=C, kernel=kernel, splitk=splitk)
    assert torch.equal(C, (A.double() @ B.double()).to(dt))


def test_auto_plan_for_shard_shapes():
    """Auto: W4 where 256x256 tiles fill the chip, T128 for the under-filled
    matrix_parallel shards (and 2048^3)."""
    def plan(M, N, K):
        A = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.empty(K, N, device="cuda", dtype=torch.bfloat16)
        return gemm.kernel_for(A, B), gemm.splitk_for(A, B)
    # >= 2 tiles per CU, K / 64 even: the streaming W4S; shared device: W4
    assert plan(16384, 16384, 16384) == ("pdmb_w4s", 1)
    assert plan(16384, 2048, 16384) == ("pdmb_w4s", 1)
    with gemm.shared_device():
        assert plan(16384, 16384, 16384) == ("pdmb_w4_nn", 1)
    assert plan(8192, 8192, 8192) == ("pdmb_w4s", 1)
    for shape in ((8192, 1024, 8192), (4096, 512, 4096), (2048, 2048, 2048), (4096, 2048, 4096)):
        k, S = plan(*shape)  # more workgroups than 256x256 tiles: a smaller tile or a split W4
        assert k in TILED[1:] or (k == "pdmb_w4_nn" and S > 1), (shape, k, S)
    assert plan(16384, 1024, 256)[1] == 1  # too little K to split
    # edge tiles: 3 waves of 256x128 beat 2 of 256x256 at 66 % busy (profiles/r2_planner_fit.jsonl)
    assert plan(3000, 7000, 5056) == ("pdmb_t256x128_nn", 1)
    assert plan(6000, 6000, 6144)[0] == "pdmb_w4_nn"


@pytest.mark.parametrize("kernel,M,N,K,splitk", [
    ("auto", 8192, 1024, 8192, 0), ("auto", 2048, 2048, 2048, 0), ("t128", 4096, 512, 4096, 2),
    ("w4", 4096, 512, 4096, 8), ("t128", 4096, 4096, 4096, 1), ("t256x128", 4096, 2048, 4096, 1),
    ("t256x128", 2048, 1024, 8192, 4), ("t128", 2560, 512, 8192, 3), ("w4", 2560, 4096, 16384, 3),
    ("t128", 1024, 256, 16384, 6), ("w4", 512, 5632, 16384, 5)])
def test_tiled_random_and_bitwise_repeatable(kernel, M, N, K, splitk):
    """Random data vs fp64, and a race screen for the LDS-DMA ring and the
    split-K meeting: the slices meet in a fixed order, so every launch is
    bitwise identical whichever slice arrives last."""
    torch.manual_seed(M + N)
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    ref = gemm.matmul(A, B, kernel=kernel, splitk=splitk)
    assert _relerr(ref, _ref(A, B)) < TOL[torch.bfloat16]
    for _ in range(30):
        assert torch.equal(gemm.matmul(A, B, kernel=kernel, splitk=splitk), ref)
    # W4 unsplit differs only by fp32 summation order
    assert _relerr(gemm.matmul(A, B, kernel="w4", splitk=1), ref.double()) < 1e-2


def test_tile_family_matches_w4_bitwise_unsplit():
    """Same per-output fp32 accumulation order (K-tiles ascending, 16x16x32 MFMA
    steps): the 128x128, 256x128 and 256x256 kernels agree bitwise."""
    torch.manual_seed(4)
    A = torch.randn(2048, 3072, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(3072, 1536, device="cuda", dtype=torch.bfloat16)
    ref = gemm.matmul(A, B, kernel="w4", splitk=1)
    for k in ("t128", "t128x2", "t256x128"):
        assert torch.equal(gemm.matmul(A, B, kernel=k, splitk=1), ref), k


@pytest.mark.experiments
@pytest.mark.parametrize("b,M,N,K", [(1, 256, 256, 64), (1, 256, 512, 128), (1, 2304, 1280, 192),
                                     (3, 1024, 768, 256), (1, 4096, 4096, 512), (1, 8192, 2048, 128)])
def test_persistent_w4_matches_w4_bitwise(b, M, N, K):
    """Persistent W4 (per-XCD work queues, stealing): same tiles, same
    accumulation order, so bitwise equal to W4 — for grids smaller than the
    chip, than 8 (XCDs with empty queues steal), and batched. Three launches
    each: the queue counters must be back at zero after every one."""
    _need("x_w4_pers")
    g = torch.Generator(device="cuda").manual_seed(b * 7 + M + N + K)
    shape = (b,) if b > 1 else ()
    A = torch.randn(*shape, M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    B = torch.randn(*shape, K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = gemm.matmul(A, B, kernel="w4", splitk=1)
    for _ in range(3):
        out = torch.full_like(ref, float("nan"))
        gemm.matmul(A, B, out=out, kernel="x_w4_pers")
        assert torch.equal(out, ref)
    assert _relerr(ref, _ref(A, B)) < TOL[torch.bfloat16]


@pytest.mark.parametrize("b,M,N,K", [(1, 256, 256, 384), (1, 2304, 1280, 384), (3, 1024, 768, 512),
                                     (1, 4096, 4096, 512), (1, 8192, 2048, 1024), (1, 16384, 8192, 384),
                                     (1, 4096, 4096, 640), (1, 2048, 16384, 384), (1, 16384, 2048, 384),
                                     (1, 1024, 32768, 384), (1, 32768, 1024, 384)])
def test_streaming_w4s_matches_w4_bitwise(b, M, N, K):
    """W4S (one K-tile stream per CU, overlapped epilogue): bitwise equal to W4
    for one tile per workgroup, several, uneven counts (T not a multiple of the
    grid), batches, and >= 2 tiles per CU under every thin-grid block->tile map
    (supertiles 2-5: 8x64, 64x8, 4x128 and 128x4 tile grids)."""
    g = torch.Generator(device="cuda").manual_seed(b * 5 + M + N + K)
    shape = (b,) if b > 1 else ()
    A = torch.randn(*shape, M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    B = torch.randn(*shape, K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = gemm.matmul(A, B, kernel="w4", splitk=1)
    for _ in range(2):
        out = torch.full_like(ref, float("nan"))
        gemm.matmul(A, B, out=out, kernel="w4s")
        assert torch.equal(out, ref)


@pytest.mark.experiments
@pytest.mark.parametrize("b,M,N,K", [(1, 4096, 4096, 512), (2, 4096, 8192, 384), (1, 8192, 8192, 384),
                                     (1, 16384, 2048, 384)])
def test_streaming_w4s_rot_matches_w4_bitwise(b, M, N, K):
    """A/B kernel x_w4s_rot (W4S with the XCD -> block position rotated per
    round, map_tile supertile 6; thin grids keep their own maps): every tile
    once, bitwise equal to W4."""
    if not gemm.experiments_built():
        pytest.skip("x_w4s_rot: PDMB_EXPERIMENTS=1 build only")
    g = torch.Generator(device="cuda").manual_seed(b * 7 + M + N + K)
    shape = (b,) if b > 1 else ()
    A = torch.randn(*shape, M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    B = torch.randn(*shape, K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = gemm.matmul(A, B, kernel="w4", splitk=1)
    out = torch.full_like(ref, float("nan"))
    gemm.matmul(A, B, out=out, kernel="x_w4s_rot")
    assert torch.equal(out, ref)


def test_streaming_w4s_fp16_exact():
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randint(-3, 4, (2048, 1024), device="cuda", generator=g).to(torch.float16)
    B = torch.randint(-3, 4, (1024, 4096), device="cuda", generator=g).to(torch.float16)
    R = (A.double() @ B.double()).to(torch.float16)
    assert torch.equal(gemm.matmul(A, B, kernel="w4s"), R)
    with pytest.raises(RuntimeError):  # K / 64 odd: W4S cannot stream it
        gemm.matmul(A[:, :960], B[:960], kernel="w4s")


@pytest.mark.experiments
def test_persistent_w4_streams_graph_and_cu_budget():
    """Queues are per stream: persistent launches on two streams at once stay
    exact; a graph replays exactly; a CU-masked stream (fewer workgroups than
    CUs) still covers every tile."""
    _need("x_w4_pers")
    from pytorch_distributed_matmul_benchmark_amd.parallel.overlap import MaskedStream

    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randint(-3, 4, (4096, 2048), device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randint(-3, 4, (2048, 4096), device="cuda", generator=g).to(torch.bfloat16)
    R = (A.double() @ B.double()).to(torch.bfloat16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty_like(R) for _ in range(6)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        with torch.cuda.stream(s1 if i % 2 else s2):
            gemm.matmul(A, B, out=o, kernel="x_w4_pers")
    torch.cuda.synchronize()
    assert all(torch.equal(o, R) for o in outs)
    s = torch.cuda.Stream()
    out = torch.empty_like(R)
    with torch.cuda.stream(s):
        gemm.matmul(A, B, out=out, kernel="x_w4_pers")  # the stream's queue exists first
    s.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        gemm.matmul(A, B, out=out, kernel="x_w4_pers")
    for _ in range(3):
        out.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, R)
    ms = MaskedStream(torch.device("cuda", 0), 24)
    try:
        out.fill_(float("nan"))
        with torch.cuda.stream(ms.stream), ms.budget():
            gemm.matmul(A, B, out=out, kernel="x_w4_pers")
        torch.cuda.synchronize()
        assert torch.equal(out, R)
    finally:
        ms.close()


def test_splitk_concurrent_streams_and_graph():
    """Per-stream counters: split-K GEMMs on two streams at once stay exact; a
    torch.cuda.graph capture of one replays exactly (counters re-zeroed by
    every launch)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randint(-3, 4, (2048, 4096), device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randint(-3, 4, (4096, 1024), device="cuda", generator=g).to(torch.bfloat16)
    R = (A.double() @ B.double()).to(torch.bfloat16)
    for kernel in ("w4", "t256x128", "t128"):
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = [torch.empty_like(R) for _ in range(8)]
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            with torch.cuda.stream(s1 if i % 2 else s2):
                gemm.matmul(A, B, out=o, kernel=kernel, splitk=4)
        torch.cuda.synchronize()
        assert all(torch.equal(o, R) for o in outs)
        s = torch.cuda.Stream()
        out = torch.empty_like(R)
        with torch.cuda.stream(s):
            gemm.matmul(A, B, out=out, kernel=kernel, splitk=4)  # counters for s exist first
        s.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            gemm.matmul(A, B, out=out, kernel=kernel, splitk=4)
        for _ in range(3):
            out.fill_(float("nan"))
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, R)


def test_splitk_graphs_from_one_stream_replay_concurrently():
    """Each capture takes its own split-K counter set (gemm_dispatch.cpp
    stream_counters): two graphs captured on ONE stream replay at the same time
    on two other streams, beside eager split-K launches on the capture stream,
    and every output stays exact."""
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randint(-3, 4, (2048, 4096), device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randint(-3, 4, (4096, 1024), device="cuda", generator=g).to(torch.bfloat16)
    R = (A.double() @ B.double()).to(torch.bfloat16)
    for kernel in ("w4", "t128"):
        s = torch.cuda.Stream()
        outs = [torch.empty_like(R) for _ in range(3)]
        with torch.cuda.stream(s):
            gemm.matmul(A, B, out=outs[2], kernel=kernel, splitk=4)
        s.synchronize()
        graphs = []
        for o in outs[:2]:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                gemm.matmul(A, B, out=o, kernel=kernel, splitk=4)
            graphs.append(gr)
        r1, r2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(5):
            for o in outs:
                o.fill_(float("nan"))
            torch.cuda.synchronize()
            with torch.cuda.stream(r1):
                graphs[0].replay()
            with torch.cuda.stream(r2):
                graphs[1].replay()
            with torch.cuda.stream(s):
                gemm.matmul(A, B, out=outs[2], kernel=kernel, splitk=4)
            torch.cuda.synchronize()
            assert all(torch.equal(o, R) for o in outs), kernel


def test_splitk_capture_pool_exhaustion_falls_back():
    """More captures than the per-device pool holds (64 sets): the later ones
    share the capture stream's own set and still replay exactly when run one
    after another (the serial-replay contract)."""
    g = torch.Generator(device="cuda").manual_seed(6)
    A = torch.randint(-3, 4, (1024, 2048), device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randint(-3, 4, (2048, 512), device="cuda", generator=g).to(torch.bfloat16)
    R = (A.double() @ B.double()).to(torch.bfloat16)
    s = torch.cuda.Stream()
    out = torch.empty_like(R)
    with torch.cuda.stream(s):
        gemm.matmul(A, B, out=out, kernel="t128", splitk=2)
    s.synchronize()
    graphs = []
    for _ in range(72):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            gemm.matmul(A, B, out=out, kernel="t128", splitk=2)
        graphs.append(gr)
    for gr in graphs[::7] + graphs[-3:]:
        out.fill_(float("nan"))
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, R)


def test_splitk_native_bench_loop_graph():
    A = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(2048, 2048, device="cuda", dtype=torch.bfloat16)
    for kernel in ("w4", "t128"):
        for graph in (False, True):
            out.zero_()
            assert gemm.bench_matmul(A, B, out, iters=5, warmup=0, graph=graph, kernel=kernel,
                                     splitk=2) > 0
            assert _relerr(out, _ref(A, B)) < TOL[torch.bfloat16]


def test_overlapping_views_are_refused_or_copied():
    """An expanded / overlapping-row input is made contiguous; an overlapping
    output is refused (never silently treated as contiguous)."""
    x = torch.randn(512, device="cuda", dtype=torch.bfloat16)
    A = x[None].expand(256, 512)  # stride(0) == 0
    B = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16)
    assert _relerr(gemm.matmul(A, B), _ref(A, B)) < TOL[torch.bfloat16]
    bad = torch.empty(256, device="cuda", dtype=torch.bfloat16)[None].expand(256, 256)
    with pytest.raises(RuntimeError):
        gemm.matmul(A.contiguous(), B, out=bad)
    C3 = torch.empty(256, 256, device="cuda", dtype=torch.bfloat16)[None].expand(2, 256, 256)
    with pytest.raises(RuntimeError):
        gemm.matmul(torch.randn(2, 256, 512, device="cuda", dtype=torch.bfloat16), B, out=C3)


def test_shipping_surface_refuses_diagnostics():
    if gemm.experiments_built():
        pytest.skip("experiment build")
    A = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
    for k in ("diag_f32_nodma", "diag_fp8_w4_nowait", "mfma256c_stamp", "x_w4_tall"):
        with pytest.raises(ValueError):
            gemm.matmul(A, A, kernel=k)
    assert _native.load().resolve(A, A, torch.empty_like(A), 20) == -1  # raw id, C++ side


def test_streaming_kernels_in_graphs():
    """W4S and fp8 W4S (persistent, no workspace or counters) capture and
    replay exactly: the native loop's hipGraph mode and torch.cuda.graph."""
    g = torch.Generator(device="cuda").manual_seed(21)
    A = torch.randint(-3, 4, (8192, 1024), device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randint(-3, 4, (1024, 8192), device="cuda", generator=g).to(torch.bfloat16)
    assert gemm.kernel_for(A, B) == "pdmb_w4s"
    R = (A.double() @ B.double()).to(torch.bfloat16)
    out = torch.empty_like(R)
    assert gemm.bench_matmul(A, B, out, iters=3, warmup=1, graph=True) > 0
    assert torch.equal(out, R)
    s = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        gemm.matmul(A, B, out=out)
    for _ in range(2):
        out.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, R)
    A8 = A.to(torch.float8_e4m3fn)
    B8 = B.t().contiguous().to(torch.float8_e4m3fn).t()
    assert gemm.kernel_for(A8, B8) == "pdmb_fp8_w4s"
    out8 = torch.empty_like(R)
    graph8 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph8, stream=s):
        gemm.matmul(A8, B8, out=out8)
    graph8.replay()
    torch.cuda.synchronize()
    assert torch.equal(out8, R)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
@pytest.mark.parametrize("M,N,K,batch,bcast", [(1500, 1024, 1000, 1, False), (700, 512, 1000, 3, False),
                                               (700, 512, 1000, 3, True), (6000, 6000, 6100, 1, False),
                                               (2048, 2048, 2049, 1, False),  # K % 64 == 1
                                               (1000, 1024, 1055, 1, False),  # K % 64 == 31
                                               (1000, 1024, 1087, 1, False)])  # K % 64 == 63
def test_padded_k_reads_b_in_place(dtype, M, N, K, batch, bcast):
    """K off the granule with an aligned B: only A is copied (zero columns K ..
    Kp); B is read in place and its rows past K come in as zeros through the
    DMA descriptors' extent — even when the memory after B's last row holds inf
    (B a view of a bigger buffer). Exact on small integers."""
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(M + N + K + batch)
    lead = (batch,) if batch > 1 else ()
    A = torch.randint(-3, 4, lead + (M, K), device="cuda", generator=g).to(dt)
    blead = () if bcast else lead
    big = torch.full(blead + (K + 37, N), float("inf"), device="cuda", dtype=dt)
    big[..., :K, :] = torch.randint(-3, 4, blead + (K, N), device="cuda", generator=g).to(dt)
    B = big[..., :K, :]
    assert gemm.kernel_for(A, B) == "pdmb_generic_nn" and gemm.padded_kernel_for(A, B) is not None
    C = gemm.matmul(A, B)
    R = torch.matmul(A.double(), B.double())
    assert torch.isfinite(C).all()
    assert torch.equal(C, R.to(dt))


@pytest.mark.parametrize("dtype", ["bfloat16", "float8_e4m3fn"])
@pytest.mark.parametrize("bcast", [False, True])
def test_batched_streaming_gemm_runs_per_element(dtype, bcast):
    """A batch whose elements each fill >= 2 waves of W4S runs as one launch per
    element (gemm_dispatch.cpp batch_split): exact on small integers, bitwise
    equal to each element computed alone, B broadcast (stride 0) included; the
    native timing loop takes the same path."""
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K, b = 8192, 4096, 1024, 3
    A = torch.randint(-1, 2, (b, M, K), device="cuda", generator=g).float()  # |C| << 256: exact in bf16
    B = torch.randint(-1, 2, ((1,) if bcast else (b,)) + (K, N), device="cuda", generator=g).float()
    if dtype == "float8_e4m3fn":
        A8 = A.to(torch.float8_e4m3fn)
        B8 = B.transpose(-1, -2).contiguous().to(torch.float8_e4m3fn).transpose(-1, -2)
    else:
        A8, B8 = A.to(torch.bfloat16), B.to(torch.bfloat16)
    if bcast:
        B8 = B8.expand(b, K, N)
    assert gemm.kernel_for(A8, B8) in ("pdmb_w4s", "pdmb_fp8_w4s")
    C = gemm.matmul(A8, B8)
    R = torch.matmul(A.double(), B.double())
    assert torch.equal(C.double(), R.expand_as(C.double()) if bcast else R)
    for i in range(b):
        assert torch.equal(gemm.matmul(A8[i], B8[i]), C[i])
    out = torch.empty_like(C)
    gemm.bench_matmul(A8, B8, out, iters=2, warmup=1)
    assert torch.equal(out, C)



# ---- 192-row tiles (round 5): T192 (192x192, B as three 64-column panels) and
# T192x128 — the grids no 256- / 128-tile cuts into whole waves -----------------
@pytest.mark.parametrize("kernel", ["t192", "t192x128"])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("b,M,N,K,splitk", [(1, 3072, 3072, 1024, 1), (1, 2304, 2304, 768, 1),
                                            (1, 192, 192, 64, 1), (1, 384, 576, 128, 1),
                                            (2, 576, 384, 320, 1), (1, 1920, 1152, 2048, 2),
                                            (1, 768, 768, 4096, 4), (1, 1000, 1048, 704, 1)])
def test_t192_exact_small_integers(kernel, dtype, b, M, N, K, splitk):
    """Exact on small integers (every fp32 partial sum exact): one and several
    tiles, batched, split-K 2 / 4 (odd K-tile counts), edge tiles in M and N
    (1000 x 1048), K of one K-tile; nothing written outside C."""
    dt = DT[dtype]
    g = torch.Generator(device="cuda").manual_seed(b * 11 + M + 3 * N + K + splitk)
    A = torch.randint(-3, 4, (b, M, K), device="cuda", generator=g).to(dt)
    B = torch.randint(-3, 4, (b, K, N), device="cuda", generator=g).to(dt)
    big = torch.full((b, M + 8, N + 24), float("nan"), device="cuda", dtype=dt)
    out = big[:, :M, :N]
    if b == 1:
        A, B, out = A[0], B[0], out[0]
    assert gemm.kernel_for(A, B, out, kernel=kernel) == f"pdmb_{kernel}_nn"
    assert gemm.splitk_for(A, B, out, kernel=kernel, splitk=splitk) == splitk
    for _ in range(2):  # split-K counters re-zeroed by every launch
        gemm.matmul(A, B, out=out, kernel=kernel, splitk=splitk)
        assert torch.equal(out, (A.double() @ B.double()).to(dt))
    assert torch.isnan(big[..., :M, N:]).all() and torch.isnan(big[..., M:, :]).all()


@pytest.mark.parametrize("kernel", ["t192", "t192x128"])
def test_t192_identity_asymmetric_and_bitwise_w4(kernel):
    """A = I with an asymmetric B (catches a column permutation of the panel
    image or the epilogue), and on random data unsplit bitwise equal to W4 (the
    same MFMA chain per output block)."""
    n = 768
    I = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    Bs = ((torch.arange(n * 1152, device="cuda").view(n, 1152) * 7) % 97).to(torch.bfloat16)
    assert torch.equal(gemm.matmul(I, Bs, kernel=kernel), Bs)
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(1536, 2048, device="cuda", dtype=torch.bfloat16, generator=g)
    B = torch.randn(2048, 1536, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = gemm.matmul(A, B, kernel="w4", splitk=1)
    assert torch.equal(gemm.matmul(A, B, kernel=kernel, splitk=1), ref)


@pytest.mark.parametrize("kernel", ["t192", "t192x128"])
def test_t192_race_screen(kernel):
    torch.manual_seed(31)
    A = torch.randn(3072, 3072, device="cuda", dtype=torch.bfloat16)
    B = torch.randn(3072, 3072, device="cuda", dtype=torch.bfloat16)
    ref = gemm.matmul(A, B, kernel=kernel)
    assert _relerr(ref, _ref(A, B)) < TOL[torch.bfloat16]
    for _ in range(20):
        assert torch.equal(gemm.matmul(A, B, kernel=kernel), ref)


def test_t192_is_auto_on_one_wave_grids():
    """3072^2 is one wave of 192x192 tiles (144 256-tiles fill 56 % of the
    CUs) and 2304^2 84 % of one of 192x128: auto takes the 192-row tiles there
    and keeps W4S / W4 where 256-tiles fill the chip."""
    mk = lambda m, n, k: (torch.empty(m, k, device="cuda", dtype=torch.bfloat16),
                          torch.empty(k, n, device="cuda", dtype=torch.bfloat16))
    assert gemm.kernel_for(*mk(3072, 3072, 3072)) == "pdmb_t192_nn"
    assert gemm.kernel_for(*mk(2304, 2304, 4096)) == "pdmb_t192x128_nn"
    assert gemm.kernel_for(*mk(16384, 16384, 16384)) == "pdmb_w4s"


@pytest.mark.experiments  # PDMB_SPLITK_PREFETCH=0: the experiments build reads it
@pytest.mark.parametrize("kernel,M,N,K,dt", [("t128", 1024, 1024, 4096, "bfloat16"), ("t128", 700, 264, 2048, "bfloat16"),
                                            ("f32_t128", 1000, 1052, 4096, "float32"),
                                            ("f32_t64", 700, 300, 2048, "float32")])
def test_split3_prefetch_bitwise(kernel, M, N, K, dt, monkeypatch):
    """Round 5: the 3-way reducer's row-ahead prefetch of both other slots
    (splitk.h splitk_load_others3; T128 and the 4-stage fp32 tiles) sums in
    slot order, so it is bitwise equal to the row-by-row reducer
    (PDMB_SPLITK_PREFETCH=0) on random data, and exact on small integers."""
    d = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g).to(d)
    B = torch.randn(K, N, device="cuda", generator=g).to(d)
    C1 = gemm.matmul(A, B, kernel=kernel, splitk=3)
    monkeypatch.setenv("PDMB_SPLITK_PREFETCH", "0")
    C0 = gemm.matmul(A, B, kernel=kernel, splitk=3)
    monkeypatch.delenv("PDMB_SPLITK_PREFETCH")
    assert torch.equal(C1, C0)
    Ai = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(d)
    Bi = torch.randint(-3, 4, (K, N), device="cuda", generator=g).to(d)
    C = gemm.matmul(Ai, Bi, kernel=kernel, splitk=3)
    assert torch.equal(C.double(), (Ai.double() @ Bi.double()).to(d).double())


# The wave-quantisation tails the SHIPPING planner picks by itself (refined
# halves / quarters for bf16 / fp16 / fp8; the split f32_t128 tail for exact
# fp32), batched grids included: exact on small integers, nothing written
# outside C.
SHIPPING_TAILS = [("bfloat16", 1, 6144, 6144, 6144), ("bfloat16", 2, 6144, 6144, 6144),
                  ("bfloat16", 1, 6000, 6000, 6144), ("bfloat16", 1, 4608, 4608, 3072),
                  ("bfloat16", 1, 3000, 7000, 5056), ("float16", 2, 6000, 5888, 3072),
                  ("float16", 1, 7168, 7168, 1024), ("float8_e4m3fn", 1, 6144, 6144, 6144),
                  ("float8_e4m3fn", 1, 6000, 6000, 6144), ("float8_e4m3fn", 2, 6000, 5888, 3072),
                  ("float32", 1, 5120, 5120, 5120), ("float32", 1, 3072, 3072, 3072),
                  ("float32", 1, 6000, 5888, 3072), ("float32", 2, 4608, 4608, 3072)]


@pytest.mark.parametrize("dtype,b,M,N,K", SHIPPING_TAILS)
def test_shipping_tail_plans_exact(dtype, b, M, N, K):
    dt = getattr(torch, dtype)
    fp8 = dt == gemm.FP8
    g = torch.Generator(device="cuda").manual_seed(M + N + K + b)
    lo, hi = (-2, 3) if fp8 else (-3, 4)
    Af = torch.randint(lo, hi, (b, M, K), device="cuda", generator=g).float()
    Bf = torch.randint(lo, hi, (b, K, N), device="cuda", generator=g).float()
    A = Af.to(dt)
    B = Bf.transpose(-1, -2).contiguous().to(dt).transpose(-1, -2) if fp8 else Bf.to(dt)
    if b == 1:
        A, B, Af, Bf = A[0], B[0], Af[0], Bf[0]
    odt = gemm.out_dtype(dt)
    big = torch.full((b, M + 16, N + 24), float("nan"), device="cuda", dtype=odt)
    out = big[:, :M, :N] if b > 1 else big[0, :M, :N]
    m1, S, t1, r = gemm.tail_split_for(A, B, out)
    assert t1 > 0 and m1 == 0 and (r > 1 or S > 1), (m1, S, t1, r)  # a tail is planned
    gemm.matmul(A, B, out=out)
    assert torch.equal(out, torch.matmul(Af.double(), Bf.double()).to(odt))
    assert torch.isnan(big[..., N:]).all() and torch.isnan(big[:, M:]).all()
