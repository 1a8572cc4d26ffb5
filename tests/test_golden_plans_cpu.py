"""Golden plans: the kernel and split-K the shipping planner chooses for every
reference-shaped GEMM, pinned (VERDICT r5 "Next #3").

Shapes (the reference's defaults, /root/reference/matmul_scaling_benchmark.py
:351-352 and :179-188, matmul_benchmark.py:157-158): the squares 4096 / 8192 /
16384; matrix_parallel's column shards n x n/ws x n at ws = 2 / 4 / 8; and
batch_parallel's local units, bmm of 2 and 4 squares (global batch 4 at ws =
2 / 1). Every dtype the CLI takes (bf16, fp16, exact fp32, fp8 e4m3 -> bf16),
planned on a device of its own (``cus = 0``: the headline and serialized
modes) and beside a collective (``cus = -1``: gemm.shared_device, the
overlapped modes). None of these plans runs a wave-quantisation tail.

A planner change that moves one of these plans must edit this table on
purpose, with the measurement that justifies it. (Round 6: exact fp32 on whole
waves of 256x256 tiles, K >= 4096, alone on the device, moved to f32_w4l:
profiles/r8y_f32_w4l_one_wave.md, r8za/.) The shipping build also
reads no A/B switch from the environment (gemm_dispatch.cpp ``ab_switch``):
setting every one of them changes no plan.
"""
import os

import pytest

from pytorch_distributed_matmul_benchmark_amd.ops import _native

DT = {"bf16": 2, "fp16": 1, "fp32": 0, "fp8": 3}

# (dtype, M, N, K, batch): (kernel alone, split, kernel beside a collective, split)
GOLDEN = {
    ("bf16", 4096, 4096, 4096, 1): ("w4_nn", 1, "w4_nn", 1),
    ("bf16", 4096, 2048, 4096, 1): ("t256x128_nn", 1, "t256x128_nn", 1),
    ("bf16", 4096, 1024, 4096, 1): ("t128_nn", 1, "t128_nn", 1),
    ("bf16", 4096, 512, 4096, 1): ("t128_nn", 2, "t128_nn", 2),
    ("bf16", 4096, 4096, 4096, 2): ("w4s", 1, "w4_nn", 1),
    ("bf16", 4096, 4096, 4096, 4): ("w4s", 1, "w4_nn", 1),
    ("bf16", 8192, 8192, 8192, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 8192, 4096, 8192, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 8192, 2048, 8192, 1): ("w4_nn", 1, "w4_nn", 1),
    ("bf16", 8192, 1024, 8192, 1): ("t256x128_nn", 1, "t256x128_nn", 1),
    ("bf16", 8192, 8192, 8192, 2): ("w4s", 1, "w4_nn", 1),
    ("bf16", 8192, 8192, 8192, 4): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 16384, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 8192, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 4096, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 2048, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 16384, 16384, 2): ("w4s", 1, "w4_nn", 1),
    ("bf16", 16384, 16384, 16384, 4): ("w4s", 1, "w4_nn", 1),
    ("fp16", 4096, 4096, 4096, 1): ("w4_nn", 1, "w4_nn", 1),
    ("fp16", 4096, 2048, 4096, 1): ("t256x128_nn", 1, "t256x128_nn", 1),
    ("fp16", 4096, 1024, 4096, 1): ("t128_nn", 1, "t128_nn", 1),
    ("fp16", 4096, 512, 4096, 1): ("t128_nn", 2, "t128_nn", 2),
    ("fp16", 4096, 4096, 4096, 2): ("w4s", 1, "w4_nn", 1),
    ("fp16", 4096, 4096, 4096, 4): ("w4s", 1, "w4_nn", 1),
    ("fp16", 8192, 8192, 8192, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 8192, 4096, 8192, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 8192, 2048, 8192, 1): ("w4_nn", 1, "w4_nn", 1),
    ("fp16", 8192, 1024, 8192, 1): ("t256x128_nn", 1, "t256x128_nn", 1),
    ("fp16", 8192, 8192, 8192, 2): ("w4s", 1, "w4_nn", 1),
    ("fp16", 8192, 8192, 8192, 4): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 16384, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 8192, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 4096, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 2048, 16384, 1): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 16384, 16384, 2): ("w4s", 1, "w4_nn", 1),
    ("fp16", 16384, 16384, 16384, 4): ("w4s", 1, "w4_nn", 1),
    ("fp32", 4096, 4096, 4096, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 4096, 2048, 4096, 1): ("f32_t128x2_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 4096, 1024, 4096, 1): ("f32_t128_nn", 1, "f32_t128_nn", 1),
    ("fp32", 4096, 512, 4096, 1): ("f32_t64_nn", 1, "f32_t64_nn", 1),
    ("fp32", 4096, 4096, 4096, 2): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 4096, 4096, 4096, 4): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 8192, 8192, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 4096, 8192, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 2048, 8192, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 1024, 8192, 1): ("f32_t128x2_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 8192, 8192, 2): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 8192, 8192, 8192, 4): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 16384, 16384, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 8192, 16384, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 4096, 16384, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 2048, 16384, 1): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 16384, 16384, 2): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp32", 16384, 16384, 16384, 4): ("f32_w4l_nn", 1, "f32_t128x2_nn", 1),
    ("fp8", 4096, 4096, 4096, 1): ("fp8_w4_nt", 1, "fp8_w4_nt", 1),
    ("fp8", 4096, 2048, 4096, 1): ("fp8_t256x128_nt", 1, "fp8_t256x128_nt", 1),
    ("fp8", 4096, 1024, 4096, 1): ("fp8_t128_nt", 1, "fp8_t128_nt", 1),
    ("fp8", 4096, 512, 4096, 1): ("fp8_t128_nt", 1, "fp8_t128_nt", 1),
    ("fp8", 4096, 4096, 4096, 2): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 4096, 4096, 4096, 4): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 8192, 8192, 8192, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 8192, 4096, 8192, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 8192, 2048, 8192, 1): ("fp8_w4_nt", 1, "fp8_w4_nt", 1),
    ("fp8", 8192, 1024, 8192, 1): ("fp8_t256x128_nt", 1, "fp8_t256x128_nt", 1),
    ("fp8", 8192, 8192, 8192, 2): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 8192, 8192, 8192, 4): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 16384, 16384, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 8192, 16384, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 4096, 16384, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 2048, 16384, 1): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 16384, 16384, 2): ("fp8_w4s", 1, "fp8_w4_nt", 1),
    ("fp8", 16384, 16384, 16384, 4): ("fp8_w4s", 1, "fp8_w4_nt", 1),
}

AB_SWITCHES = {"PDMB_SPLIT3": "0", "PDMB_SPLIT56": "0", "PDMB_SPLIT8": "0", "PDMB_SPLIT3_SMALL": "0",
               "PDMB_SPLIT_SLOT_LAT": "0", "PDMB_F32T64": "0", "PDMB_F32T64X2": "0",
               "PDMB_F32T64X2_FULL": "0", "PDMB_F32X2SPLIT": "0", "PDMB_T192": "0",
               "PDMB_TILE_TAIL": "4", "PDMB_TAIL_REFINE": "2", "PDMB_STREAMK": "1",
               "PDMB_TAIL_DP_W4S": "1", "PDMB_SPLITK_PREFETCH": "0"}


@pytest.fixture(scope="module")
def C():
    try:
        mod = _native.load(build_if_missing=False)
    except Exception as e:  # pragma: no cover - the build check runs first
        pytest.skip(f"native extension not built: {e}")
    if mod.EXPERIMENTS:
        pytest.skip("a PDMB_EXPERIMENTS=1 build reads the A/B switches: golden plans pin the shipping build")
    return mod


def _plan(C, dt, M, N, K, b, cus):
    k, S, _cost, m1, tS, t1, r = C.plan_shape(DT[dt], M, N, K, b, 0, cus)
    return C.kernel_name(k).replace("pdmb_", ""), S, (m1, tS, t1, r)


def _all(C):
    out = {}
    for (dt, M, N, K, b) in GOLDEN:
        k0, s0, t0 = _plan(C, dt, M, N, K, b, 0)
        k1, s1, t1 = _plan(C, dt, M, N, K, b, -1)
        out[(dt, M, N, K, b)] = (k0, s0, k1, s1, t0, t1)
    return out


def test_golden_plans(C):
    got = _all(C)
    moved = {key: (got[key][:4], want) for key, want in GOLDEN.items() if got[key][:4] != want}
    assert not moved, f"plans moved (got, pinned): {moved}"
    assert all(v[4] == (0, 1, 0, 1) and v[5] == (0, 1, 0, 1) for v in got.values())


def test_shipping_planner_ignores_the_ab_switches(C, monkeypatch):
    """Every A/B switch set to its 'rule off' / forcing value: the reference
    shapes, a 3-way-split grid (2560 x 4096 x 16384) and a wave-tail grid
    (6144^3) plan exactly as without them."""
    extra = [("bf16", 2560, 4096, 16384, 1), ("bf16", 6144, 6144, 6144, 1), ("fp8", 6144, 6144, 6144, 1),
             ("fp32", 2560, 256, 8192, 1), ("fp32", 5120, 5120, 5120, 1)]
    before = _all(C)
    before_x = {s: (_plan(C, *s, 0), _plan(C, *s, -1)) for s in extra}
    for k, v in AB_SWITCHES.items():
        monkeypatch.setenv(k, v)
    assert _all(C) == before
    assert {s: (_plan(C, *s, 0), _plan(C, *s, -1)) for s in extra} == before_x
