"""The C++ GEMM planner (gemm_dispatch.cpp plan / resolve_kernel) queried by
SHAPE on CPU (bindings plan_shape: aligned stand-in operands, no GPU needed):
which kernel and split-K auto picks for the reference's shapes, per dtype.

Shapes: square sizes (matmul_benchmark.py:157-158), matrix_parallel column
shards at ws = 2 / 4 / 8 (matmul_scaling_benchmark.py:179-188 at :351-352)."""
import pytest

from pytorch_distributed_matmul_benchmark_amd.ops import _native

F32, F16, BF16, FP8 = 0, 1, 2, 3


@pytest.fixture(scope="module")
def C():
    try:
        return _native.load(build_if_missing=False)
    except Exception as e:  # pragma: no cover - the build check runs first
        pytest.skip(f"native extension not built: {e}")


def ab(C, monkeypatch, name, value) -> bool:
    """Set one of the planner's A/B switches; True if this build reads it. Only
    a PDMB_EXPERIMENTS=1 build does (gemm_dispatch.cpp ab_switch): in the
    shipping build the rule stays on, so the "switch off" halves below run
    on experiment builds only (tests/test_golden_plans_cpu.py checks that the
    shipping build ignores every switch)."""
    monkeypatch.setenv(name, value)
    return bool(C.EXPERIMENTS)


def plan(C, dt, M, N, K, b=1, kernel=0, cus=0):
    k, S, cost, m1, tS, t1, r = C.plan_shape(dt, M, N, K, b, kernel, cus)
    return C.kernel_name(k), S, cost, (m1, tS, t1, r)


@pytest.mark.parametrize("n", [4096, 8192, 16384])
@pytest.mark.parametrize("ws", [2, 4, 8])
def test_f32_shards_fill_the_chip(C, n, ws):
    """Exact-fp32 shards never run a grid that leaves most CUs idle: the chosen
    plan's workgroups (tiles x split) cover >= 3/4 of the 256 CUs or at least a
    wave, and the under-filled 4096 shards go to the small tile or a split W4."""
    shard = n // ws
    k, S, cost, _ = plan(C, F32, n, shard, n)
    bm, bn = {"pdmb_f32_t128_nn": (128, 128), "pdmb_f32_t128x2_nn": (128, 128),
              "pdmb_f32_t64_nn": (64, 128), "pdmb_f32_t64x2_nn": (64, 128)}.get(k, (256, 256))
    units = -(-n // bm) * -(-shard // bn) * max(S, 1)
    assert units >= 192, (n, ws, k, S)
    if n == 4096:
        assert k in ("pdmb_f32_t128_nn", "pdmb_f32_t128x2_nn", "pdmb_f32_t64_nn", "pdmb_f32_t64x2_nn") or (
            k == "pdmb_f32_w4_nn" and S > 1)


def test_f32_full_grids_take_two_128_tiles_per_cu(C):
    """Full fp32 grids beside a collective run f32_t128x2 (measured ahead of
    f32_256s at 4k / 8k / 16k in the same process, profiles/r3i_f32_256p_ab.jsonl);
    whole waves of 256x256 tiles alone on the device, K >= 4096, run the lean
    W4 loop (round 6, f32_w4l: +0.5 % median over f32_t128x2, profiles/r8za/,
    r8y/); partial waves and short K keep f32_t128x2."""
    for n in (4096, 8192, 16384):
        assert plan(C, F32, n, n, n)[:2] == ("pdmb_f32_w4l_nn", 1)
        assert plan(C, F32, n, n, n, cus=-1)[0] == "pdmb_f32_t128x2_nn"
    assert plan(C, F32, 4096, 4096, 4096, b=2)[0] == "pdmb_f32_w4l_nn"
    assert plan(C, F32, 4096, 4096, 4128)[0] == "pdmb_f32_w4l_nn"  # 129 K-tiles: the loop takes any count
    for shape in ((4352, 3840, 4096), (4096, 2048, 4096), (4096, 4096, 2048), (16384, 16384, 1024),
                  (6144, 6144, 6144), (10240, 10240, 10240)):
        assert plan(C, F32, *shape)[0] != "pdmb_f32_w4l_nn", shape


def test_f32_planner_prefers_cheaper_plan(C):
    """Whatever auto picks costs (model) within the planner's 3 % hysteresis of
    forcing W4 or T128 (an incumbent is only replaced by a clear win)."""
    for shape in ((4096, 512, 4096), (4096, 1024, 4096), (4096, 2048, 4096), (2048, 2048, 2048),
                  (1000, 1052, 4096), (8192, 1024, 8192), (6144, 6144, 6144)):
        auto = plan(C, F32, *shape)
        for forced in (29, 51, 53):
            f = plan(C, F32, *shape, kernel=forced)
            assert auto[2] <= f[2] / 0.97 + 1e-6, (shape, auto, f)
    # the measured winners on the under-filled shards (profiles/r3_f32_t128x2_ab.jsonl):
    # two 128x128 workgroups per CU where the grid has two per CU, else one
    assert plan(C, F32, 4096, 2048, 4096)[0] == "pdmb_f32_t128x2_nn"
    for shape in ((4096, 1024, 4096), (2048, 2048, 2048)):
        assert plan(C, F32, *shape)[0] == "pdmb_f32_t128_nn"


def test_f32_two_per_cu_tile_needs_two_per_cu(C):
    """f32_t128x2 (2-stage ring, two workgroups per CU) is never planned on a
    grid that leaves CUs with one workgroup (its ring is too shallow alone)."""
    for shape in ((4096, 1024, 4096), (2048, 2048, 2048), (4096, 512, 4096), (1000, 1052, 4096),
                  (4096, 2048, 4096), (8192, 4096, 8192), (6144, 6144, 6144)):
        k, S, _, _ = plan(C, F32, *shape)
        if k == "pdmb_f32_t128x2_nn":
            assert -(-shape[0] // 128) * -(-shape[1] // 128) * max(S, 1) >= 512, (shape, S)


def test_bf16_plans(C):
    assert plan(C, BF16, 16384, 16384, 16384)[0] == "pdmb_w4s"
    assert plan(C, BF16, 16384, 16384, 16384, cus=-1)[0] == "pdmb_w4_nn"  # shared device
    k, S, _, _ = plan(C, BF16, 4096, 512, 4096)
    assert k in ("pdmb_t128_nn", "pdmb_t256x128_nn", "pdmb_t128x2_nn") or S > 1
    m1, tS, t1, r = plan(C, BF16, 6144, 6144, 6144)[3]  # wave-quantisation tail: rows, or
    assert (m1 > 0 or t1 > 0) and (tS > 1 or r > 1)       # (round 4) whole tile waves + split / refined


def test_fp8_plans(C):
    assert plan(C, FP8, 16384, 16384, 16384)[0] == "pdmb_fp8_w4s"
    assert plan(C, FP8, 4096, 512, 4096)[0].startswith("pdmb_fp8_")


def test_explicit_two_per_cu_fp32_tile_runs_any_grid(C):
    """An explicit f32_t128x2 request gets a runnable plan (split >= 1) even on a
    grid auto would not give it (one 128x128 tile, K = 32: a GPU test shape)."""
    for shape in ((256, 256, 32), (128, 128, 64), (4096, 512, 4096)):
        k, S, _, _ = plan(C, F32, *shape, kernel=53)
        assert k == "pdmb_f32_t128x2_nn" and S >= 1, (shape, k, S)


def test_refined_tail_plans(C, monkeypatch):
    """The refined wave-quantisation tail (round 4): whole waves of 256^2 tiles,
    then the last partial wave in 256x128 halves / 128x128 quarters, unsplit —
    taken over the split-K forms wherever it beats the single launch (the
    same-process A/B in profiles/r4k_*_refined_tail_ab.jsonl); PDMB_TAIL_REFINE=0
    falls back to the split-K tile-range form; stream-K only when forced."""
    monkeypatch.delenv("PDMB_TAIL_REFINE", raising=False)
    monkeypatch.delenv("PDMB_STREAMK", raising=False)
    FP8 = 3
    assert plan(C, BF16, 6144, 6144, 6144)[3] == (0, 1, 512, 4)
    assert plan(C, BF16, 7168, 7168, 7168)[3] == (0, 1, 768, 4)   # not the S = 8 split
    assert plan(C, FP8, 6144, 6144, 6144)[3] == (0, 1, 512, 4)
    assert plan(C, FP8, 4608, 4608, 3072)[3] == (0, 1, 256, 2)
    assert plan(C, BF16, 16384, 16384, 16384)[3] == (0, 1, 0, 1)  # whole waves: one launch
    if ab(C, monkeypatch, "PDMB_TAIL_REFINE", "0"):
        k, _, _, (m1, S, t1, r) = plan(C, BF16, 6144, 6144, 6144)
        # without the refined tail: the split-K tail over W4, or (round 5) one
        # launch of 192x192 tiles — 6144^3 is exactly 4 waves of them
        assert r == 1 and ((S > 1 and (m1 > 0 or t1 > 0)) or (k == "pdmb_t192_nn" and (m1, t1) == (0, 0)))
        monkeypatch.delenv("PDMB_TAIL_REFINE")
        monkeypatch.setenv("PDMB_STREAMK", "1")
        m1, S, t1, r = plan(C, FP8, 5120, 5120, 5120)[3]
        assert (m1, t1, r) == (0, 0, 0) and S == 2


def test_f32_tail_plans(C, monkeypatch):
    """Exact fp32's tail: whole two-per-CU waves of 128^2 tiles, then the rest
    split-K as one f32_t128 wave, where the light last wave would idle most CUs
    (profiles/r5g_f32_tail_ab.jsonl); none on whole waves or a full last wave."""
    monkeypatch.delenv("PDMB_TILE_TAIL", raising=False)
    F32 = 0
    assert plan(C, F32, 5120, 5120, 5120)[3] == (0, 4, 1536, 1)
    assert plan(C, F32, 3072, 3072, 3072)[3] == (0, 4, 512, 1)
    assert plan(C, F32, 16384, 16384, 16384)[3] == (0, 1, 0, 1)
    assert plan(C, F32, 6144, 6144, 6144)[3] == (0, 1, 0, 1)   # last wave half full: no split pays
    if ab(C, monkeypatch, "PDMB_TILE_TAIL", "0"):
        assert plan(C, F32, 5120, 5120, 5120)[3] == (0, 1, 0, 1)


def test_plan_report_script(C, monkeypatch):
    """scripts/plan_report.py: the planner's choice and tail form per shape."""
    import importlib.util
    import os

    monkeypatch.delenv("PDMB_TAIL_REFINE", raising=False)
    monkeypatch.delenv("PDMB_STREAMK", raising=False)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "plan_report.py")
    spec = importlib.util.spec_from_file_location("plan_report", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rows = mod.report(C, "bfloat16", [(6144, 6144, 6144), (16384, 16384, 16384)])
    assert rows[0]["tail"] == "tiles 512 / refined x4" and rows[0]["kernel"] == "pdmb_w4s"
    assert rows[1]["tail"] == "-"
    assert mod.report(C, "float32", [(5120, 5120, 5120)])[0]["tail"] == "tiles 1536 / split 4"
    assert mod.tail_form(2048, 2, 0, 1) == "rows 2048 / split 2"


def test_f32_long_k_one_wave_runs_256s(C):
    """Exactly one wave of 256x256 tiles on a long K runs the 8-wave f32_256s
    (measured 0.1-1.6 % ahead of f32_t128x2 there, profiles/r6g_f32_long_k_rule_ab.jsonl);
    shorter K or more waves keep f32_t128x2. Round 6: the lean W4 loop (f32_w4l)
    takes every such one-wave grid of whole tiles (8192 x 2048 x 8192 153.1 vs
    149.8, 4096^2 x 16384 153.3 vs 149.9 TF, profiles/r8r/); f32_256s keeps
    the edge-tile ones."""
    assert plan(C, 0, 1024, 16384, 16384)[0] == "pdmb_f32_w4l_nn"
    assert plan(C, 0, 4096, 4096, 14336)[0] == "pdmb_f32_w4l_nn"
    assert plan(C, 0, 4096, 4096, 14336, cus=-1)[0] == "pdmb_f32_t128x2_nn"
    assert plan(C, 0, 8192, 8192, 28672)[0] == "pdmb_f32_w4l_nn"  # four whole waves
    assert plan(C, 0, 8192, 8192, 28672, cus=-1)[0] == "pdmb_f32_t128x2_nn"


def test_t192_plans(C, monkeypatch):
    """Round 5: the 192-row tiles where no 256- / 128-tile cuts the grid into
    whole waves (3072^2: one wave of 192x192; 2304^2: 84 % of one of 192x128;
    measured 1260 / 1078 TF vs hipBLASLt 1067 / 965, profiles/r7e_t192_ab_bf16.jsonl),
    W4S / W4 where 256-tiles fill the chip, and PDMB_T192=0 leaves them out."""
    monkeypatch.delenv("PDMB_T192", raising=False)
    assert plan(C, BF16, 3072, 3072, 3072)[0] == "pdmb_t192_nn"
    assert plan(C, BF16, 2304, 2304, 4096)[0] == "pdmb_t192x128_nn"
    assert plan(C, FP8, 3072, 3072, 3072)[0] == "pdmb_fp8_t192_nt"
    assert plan(C, BF16, 16384, 16384, 16384)[0] == "pdmb_w4s"
    assert plan(C, BF16, 8192, 8192, 8192)[0] == "pdmb_w4s"
    if ab(C, monkeypatch, "PDMB_T192", "0"):
        assert "192" not in plan(C, BF16, 3072, 3072, 3072)[0]
        assert "192" not in plan(C, FP8, 2304, 2304, 4096)[0]


def test_fp8_short_k_streams(C):
    """Round 6: fp8 W4S down to four K-tiles (K = 512, the K4 form), measured
    1.15x fp8 W4 and at hipBLASLt's rate on the write-bound short-K grids
    (profiles/r8d/ab_fp8_k512_summary.jsonl); one tile per CU keeps W4, two
    K-tiles cannot stream."""
    FP8 = 3
    for shape in ((16384, 16384, 512), (8192, 8192, 512), (16384, 8192, 512), (16384, 16384, 1024)):
        assert plan(C, FP8, *shape)[0] == "pdmb_fp8_w4s", shape
    assert plan(C, FP8, 4096, 4096, 512)[0] == "pdmb_fp8_w4_nt"
    assert plan(C, FP8, 8192, 8192, 256)[0] != "pdmb_fp8_w4s"


def test_t192x128_multi_wave_rate(C, monkeypatch):
    """T192x128 is priced slower per K-tile past one wave (kModels kt2; measured
    0.65-0.67 us vs 0.61 on one wave, profiles/r7j_t192_ab_bf16.jsonl): the two
    two-wave grids where it lost 7-8 % to W4 go back to W4, one-wave grids keep it."""
    monkeypatch.delenv("PDMB_T192", raising=False)
    for shape in ((1024, 9216, 16384), (2560, 4608, 16384)):
        assert "192" not in plan(C, BF16, *shape)[0], shape
    for shape in ((2048, 2304, 4096), (3072, 1536, 4096), (4608, 1024, 4096)):
        assert plan(C, BF16, *shape)[0] == "pdmb_t192x128_nn", shape


def test_f32_t64_plans(C):
    """Round 5: the 64x128 exact-fp32 tile where 128x128 tiles fill the chip
    only by splitting K (4096 x 512 x 4096, the ws = 8 shard at 4k: 256 tiles
    unsplit; 2048 x 1024 x 2048) — measured ahead of f32_t128 there
    (profiles/r7p_f32_t64_ab.jsonl) — and never where f32_t128 runs a whole wave."""
    assert plan(C, F32, 4096, 512, 4096)[:2] == ("pdmb_f32_t64_nn", 1)
    assert plan(C, F32, 2048, 1024, 2048)[0] == "pdmb_f32_t64_nn"
    for shape in ((4096, 1024, 4096), (2048, 2048, 2048), (8192, 512, 8192), (8192, 1024, 8192)):
        assert plan(C, F32, *shape)[0] != "pdmb_f32_t64_nn", shape


def test_split3_plans(C, monkeypatch):
    """Round 5: the 3-way split-K, priced after the power-of-two splits and
    taken only by a clear win with >= 32 K-tiles per slice (and not on the
    256^2 fp32 tile): measured ahead on these grids (profiles/r7r_split3_ab_*.jsonl),
    left out where it lost (bf16 1024^2 x 4096, fp32 2560 x 2048 x 4096)."""
    monkeypatch.delenv("PDMB_SPLIT3", raising=False)
    assert plan(C, BF16, 2560, 4096, 16384)[:2] == ("pdmb_w4_nn", 3)
    assert plan(C, BF16, 5120, 2048, 16384)[:2] == ("pdmb_w4_nn", 3)
    assert plan(C, BF16, 1024, 1024, 4096)[1] != 3
    if ab(C, monkeypatch, "PDMB_F32T64X2", "0"):  # (f32_t64x2 takes 1536^2 x 4096 since)
        assert plan(C, F32, 2560, 256, 8192)[1] == 3
        assert plan(C, F32, 1536, 1536, 4096)[1] == 3
        assert plan(C, F32, 2560, 2048, 4096)[1] != 3
        monkeypatch.setenv("PDMB_SPLIT3", "0")
        assert plan(C, BF16, 2560, 4096, 16384)[1] != 3


def test_split56_fp32_only(C, monkeypatch):
    """Round 5: 5- / 6-way splits for exact fp32 only (measured ahead on six
    fp32 grids, mixed on bf16; profiles/r7u_split56_ab_*.jsonl)."""
    monkeypatch.delenv("PDMB_SPLIT56", raising=False)
    assert plan(C, F32, 512, 6400, 16384)[1] in (5, 6)
    assert plan(C, BF16, 2560, 256, 16384)[1] not in (5, 6)
    if ab(C, monkeypatch, "PDMB_SPLIT8", "0"):  # (8 ways takes the first grid since, test_split8_*)
        assert plan(C, F32, 1024, 256, 16384)[1] in (5, 6)
        monkeypatch.setenv("PDMB_SPLIT56", "0")
        assert plan(C, F32, 1024, 256, 16384)[1] not in (5, 6)


def test_split8_fp32_only(C, monkeypatch):
    """Round 5: the 8-way split under the 5- / 6-way rule (exact fp32 only,
    >= 32 K-tiles per slice): 1024 x 256 x 16384 on f32_t64 x 8 ran 81.5 us vs
    96.9 at 6 ways (profiles/r7ad_f32_small_split_arms.jsonl); PDMB_SPLIT8=0
    leaves it out; bf16 / fp8 auto never splits 8 ways."""
    monkeypatch.delenv("PDMB_SPLIT8", raising=False)
    assert plan(C, F32, 1024, 256, 16384)[:2] == ("pdmb_f32_t64_nn", 8)
    assert plan(C, F32, 1024, 256, 4096)[1] != 8  # 16 K-tiles per slice
    for dt in (BF16, FP8):
        for shape in ((1024, 256, 16384), (256, 256, 16384), (2048, 1024, 16384)):
            assert plan(C, dt, *shape)[1] != 8, (dt, shape)
    if ab(C, monkeypatch, "PDMB_SPLIT8", "0"):
        assert plan(C, F32, 1024, 256, 16384)[1] != 8


def test_f32_x2_split_on_small_grids(C, monkeypatch):
    """Round 5: f32_t128x2 split into >= 3 slices per CU on a grid of fewer than
    two 128x128 tiles per CU (2560 x 2048 x 4096: 320 tiles x 4 ran 303.6 us vs
    324.0 for f32_t128 x 4, profiles/r7ad_f32_small_split_arms.jsonl), never
    2 or fewer slices per CU there; an explicit f32_t128x2 request gets auto's
    split (the launch re-plans with the kernel fixed); PDMB_F32X2SPLIT=0 turns
    it off."""
    monkeypatch.delenv("PDMB_F32X2SPLIT", raising=False)
    if ab(C, monkeypatch, "PDMB_F32T64X2", "0"):  # (f32_t64x2 takes 2560 x 2048 x 4096 since)
        assert plan(C, F32, 2560, 2048, 4096)[:2] == ("pdmb_f32_t128x2_nn", 4)
        assert plan(C, F32, 2560, 2048, 4096, kernel=53)[:2] == ("pdmb_f32_t128x2_nn", 4)
        for shape in ((4096, 1024, 4096), (2048, 2048, 2048), (1536, 1536, 4096), (768, 9216, 4096),
                      (512, 12288, 4096), (1536, 5120, 4096), (2560, 512, 8192)):
            k, S, _, _ = plan(C, F32, *shape)
            tiles = -(-shape[0] // 128) * -(-shape[1] // 128)
            if k == "pdmb_f32_t128x2_nn" and tiles < 512:
                assert S > 1 and tiles * S >= 768, (shape, S)
        monkeypatch.setenv("PDMB_F32X2SPLIT", "0")
        assert plan(C, F32, 2560, 2048, 4096)[0] == "pdmb_f32_t128_nn"


def test_split_slot_latency_small_bf16_grids(C, monkeypatch):
    """Round 5: bf16 / fp16 grids of <= 64 tiles split >= 4 ways into short
    slices pay a reducer latency the slab term misses; with it, auto moves
    1024^2 x 8192 / 512 x 2048 x 8192 / 768^2 x 8192 from T128 x 4 to x 3
    (+14-17 %, profiles/r7aj_*_split_slot_latency_ab.jsonl); off with
    PDMB_SPLIT_SLOT_LAT=0; fp32 plans unchanged (fp8 T128 has it too, r7am)."""
    monkeypatch.delenv("PDMB_SPLIT_SLOT_LAT", raising=False)
    for dt in (BF16, F16):
        for shape in ((1024, 1024, 8192), (512, 2048, 8192), (768, 768, 8192)):
            assert plan(C, dt, *shape)[:2] == ("pdmb_t128_nn", 3), (dt, shape)
    other = {(F32, s): plan(C, F32, *s)[:2] for s in ((1024, 1024, 8192), (512, 512, 8192))}
    if ab(C, monkeypatch, "PDMB_SPLIT_SLOT_LAT", "0"):
        assert plan(C, BF16, 1024, 1024, 8192)[:2] == ("pdmb_t128_nn", 4)
        assert other == {(dt, s): plan(C, dt, *s)[:2] for (dt, s) in other}


def test_split3_small_bf16_grids(C, monkeypatch):
    """Round 5: T128 x 3 on bf16 / fp16 grids of <= 36 tiles below the 32
    K-tiles-per-slice minimum (its reducer prefetches both other slots;
    profiles/r7aj_*, r7ak_*); PDMB_SPLIT3_SMALL=0 restores the minimum; not on
    grids of more tiles; fp8 T128 from 16 K-tiles per slice."""
    monkeypatch.delenv("PDMB_SPLIT3_SMALL", raising=False)
    for dt in (BF16, F16):
        assert plan(C, dt, 768, 768, 4096)[:2] == ("pdmb_t128_nn", 3)
    assert plan(C, BF16, 1024, 1024, 4096)[1] != 3  # 64 tiles: mixed, left out
    assert plan(C, FP8, 768, 768, 4096)[1] != 3  # 11 fp8 K-tiles per slice: lost (r7am)
    assert plan(C, FP8, 768, 768, 8192)[:2] == ("pdmb_fp8_t128_nt", 3)  # 22: ahead
    if ab(C, monkeypatch, "PDMB_SPLIT3_SMALL", "0"):
        assert plan(C, BF16, 768, 768, 4096)[1] != 3


def test_f32_t64x2_plans(C, monkeypatch):
    """Round 5: f32_t64x2 (the 64x128 exact-fp32 tile on 2 stages, two per CU),
    split, on fp32 grids of fewer than two 128x128 tiles per CU: auto vs
    PDMB_F32T64X2=0 on 21 grids, median +6.1 %, up to +37 %
    (profiles/r7ap_f32_t64x2_auto_ab.jsonl); the full grids keep their plans
    (5120^3: f32_t128x2 waves + split tail)."""
    monkeypatch.delenv("PDMB_F32T64X2", raising=False)
    assert plan(C, F32, 1536, 3072, 1024)[:2] == ("pdmb_f32_t64x2_nn", 2)
    assert plan(C, F32, 1536, 1536, 4096)[:2] == ("pdmb_f32_t64x2_nn", 4)
    assert plan(C, F32, 1536, 3072, 1024, kernel=65)[:2] == ("pdmb_f32_t64x2_nn", 2)  # fixed = auto's
    for shape in ((4096, 4096, 4096), (8192, 8192, 8192), (16384, 16384, 16384), (16384, 1024, 16384)):
        assert plan(C, F32, *shape)[0] != "pdmb_f32_t64x2_nn", shape
    assert plan(C, F32, 5120, 5120, 5120)[3] == (0, 4, 1536, 1)  # its split tail stays
    # full grids without a split tail: split 2 ways (r7as), never unsplit
    assert plan(C, F32, 4608, 4608, 4096)[:2] == ("pdmb_f32_t64x2_nn", 2)
    assert plan(C, F32, 3072, 3584, 4096)[1] != 1 or plan(C, F32, 3072, 3584, 4096)[0] != "pdmb_f32_t64x2_nn"
    # round 6: never on the hysteresis alone — the grids where f32_t128x2 x 3 is
    # priced cheaper (and measured 2 % ahead, r7at) keep it
    for shape in ((3072, 3584, 4096), (3584, 3072, 4096), (3072, 3584, 16384)):
        assert plan(C, F32, *shape)[:2] == ("pdmb_f32_t128x2_nn", 3), shape
    if ab(C, monkeypatch, "PDMB_F32T64X2_FULL", "0"):
        assert plan(C, F32, 4608, 4608, 4096)[0] != "pdmb_f32_t64x2_nn"
        monkeypatch.setenv("PDMB_F32T64X2", "0")
        assert plan(C, F32, 1536, 3072, 1024)[0] != "pdmb_f32_t64x2_nn"
