"""Pure-Python unit tests: FLOP/TFLOPS/efficiency formulas and work partitioning."""
import pytest
import torch

from pytorch_distributed_matmul_benchmark_amd.parallel import partition as P
from pytorch_distributed_matmul_benchmark_amd.utils import metrics as M


def test_flops_match_reference_readme():
    # README.md:56-58: 0.14 / 1.10 / 8.80 TFLOP per op for 4k / 8k / 16k.
    assert round(M.square_flops(4096) / 1e12, 2) == 0.14
    assert round(M.square_flops(8192) / 1e12, 2) == 1.10
    assert round(M.square_flops(16384) / 1e12, 2) == 8.80
    assert M.gemm_flops(2, 3, 4, batch=5) == 2 * 2 * 3 * 4 * 5


def test_calculate_tflops_reference_formula():
    # matmul_scaling_benchmark.py:63-67: 2·N³·num_ops / t / 1e12
    assert M.calculate_tflops(1000, 1.0) == pytest.approx(2e9 / 1e12)
    assert M.calculate_tflops(1000, 0.5, num_ops=4) == pytest.approx(4 * 2e9 / 0.5 / 1e12)
    assert M.calculate_tflops(1000, 0.0) == 0.0


def test_peak_table():
    mi = M.peak_for_device("AMD Instinct MI355X", "gfx950:sramecc+:xnack-")
    assert mi is M.PEAKS["mi355x"]
    assert mi.for_dtype(torch.bfloat16) == pytest.approx(2516.6)
    assert mi.for_dtype(torch.float32) == pytest.approx(157.3)
    assert M.peak_for_device("", "gfx950") is M.PEAKS["mi355x"]
    assert M.peak_for_device("NVIDIA RTX 6000 Ada Generation").for_dtype(torch.float16) == 182.2
    assert M.peak_for_device("AMD Radeon RX 7900 XTX").for_dtype(torch.float32) == 61.4
    assert M.peak_for_device("Some other GPU") is None
    assert M.percent_of_peak(1258.3, mi, torch.bfloat16) == pytest.approx(50.0, rel=1e-3)


def test_efficiencies():
    assert M.scaling_efficiency(2000.0, 2, 1000.0) == pytest.approx(100.0)
    assert M.scaling_efficiency(1700.0, 2, 1000.0) == pytest.approx(85.0)
    assert M.scaling_efficiency(1.0, 2, 0.0) is None
    # reference independent-mode "scaling efficiency" = sum / (rank0 * ws)
    assert M.balance_efficiency(290.0, 140.0, 2) == pytest.approx(290 / 280 * 100)
    # compute / total, never > 100 (the backup formula was inverted, Q8)
    assert M.overlap_efficiency(6.0, 8.0) == pytest.approx(75.0)
    assert M.overlap_efficiency(9.0, 8.0) == pytest.approx(100.0)


@pytest.mark.parametrize("ws", [1, 2, 3, 4, 5, 6, 7, 8])
def test_global_batch_never_empty(ws):
    gb = P.global_batch(ws, 4)
    assert gb % ws == 0 and gb >= 4 and gb >= ws
    assert P.local_batch(ws, 4) == gb // ws >= 1
    # default matches the reference where the reference is well-defined
    if ws in (1, 2, 4):
        assert gb == 4


def test_global_batch_custom():
    assert P.global_batch(8, 16) == 16
    assert P.global_batch(3, 4) == 6
    with pytest.raises(ValueError):
        P.global_batch(0)


@pytest.mark.parametrize("n,ws", [(16384, 8), (300, 3), (100, 8), (7, 4), (4096, 1), (10, 3)])
def test_column_shards_cover_exactly(n, ws):
    shards = [P.column_shard(n, ws, r) for r in range(ws)]
    assert len({s.padded for s in shards}) == 1  # uniform gather size
    covered = []
    for s in shards:
        assert 0 <= s.width <= s.padded
        covered.extend(range(s.start, s.stop))
    assert covered == list(range(n))


def test_column_shard_alignment():
    s = P.column_shard(300, 3, 0, align=8)
    assert s.padded == 104 and s.width == 104
    last = P.column_shard(300, 3, 2, align=8)
    assert last.start == 208 and last.width == 92
    with pytest.raises(ValueError):
        P.column_shard(10, 2, 2)


@pytest.mark.parametrize("m,chunks", [(16384, 4), (300, 4), (256, 8), (1, 3), (1000, 1)])
def test_row_chunks(m, chunks):
    rc = P.row_chunks(m, chunks)
    assert rc[0][0] == 0 and rc[-1][1] == m
    assert all(a[1] == b[0] for a, b in zip(rc, rc[1:]))
    assert len(rc) <= max(chunks, 1)
    assert all(s % 256 == 0 for s, _ in rc)

