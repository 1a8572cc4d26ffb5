"""Static checks of the generated gfx950 code (CPU only: hipcc cross-compiles).

Guards the properties the kernels' performance depends on, so a source edit
that silently de-pipelines them fails here instead of on the GPU:
no register spills, the intended occupancy, exactly one vmcnt(0) drain (after
the K-loop) in the LDS-DMA kernels, and the MFMA / LDS-DMA instruction mix."""
import os
import re
import shutil
import subprocess

import pytest
from asm_cache import gfx950_asm

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_distributed_matmul_benchmark_amd", "ops", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")


def _kernels(src, tmp_path=None, experiments=False):
    """Kernels of ``src`` (default build, or with the A/B experiment kernels);
    one compile per source and flavour per test process (asm_cache.py)."""
    s = gfx950_asm(src, experiments)
    out = {}
    for m in re.finditer(r"^([A-Za-z_][\w.$]*):\s*;\s*@", s, re.M):
        name = m.group(1)
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        i = s.find(f".amdhsa_kernel {name}")
        kd = s[i:s.find(".end_amdhsa_kernel", i)]
        vg = int(re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s).group(1))
        out[name] = dict(body=body, vgpr=vg,
                         spill=int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", kd).group(1)),
                         lds=int(re.search(r"\.amdhsa_group_segment_fixed_size (\d+)", kd).group(1)))
    return out


def _loops(body, min_mfma=1):
    """(label, text) of every back edge's span (a branch to a label above it)
    holding at least ``min_mfma`` MFMA instructions."""
    lines = body.split("\n")
    lab = {}
    out = []
    for i, line in enumerate(lines):
        m = re.match(r"(\.LBB\w+):", line)
        if m:
            lab[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+ (\.LBB\w+)", line)
        if m and lab.get(m.group(1), i) < i:
            text = "\n".join(lines[lab[m.group(1)]:i])
            if len(re.findall(r"v_mfma", text)) >= min_mfma:
                out.append((m.group(1), text))
    return out


def test_bf16_lds_dma_kernel_stays_pipelined(tmp_path):
    ks = _kernels("gemm_mfma256.hip", tmp_path, experiments=True)  # SCHED 2 is an A/B build
    main = [k for k in ks if "gemm256_nn" in k and "ILi2ELi2ELb0E" in k]
    assert main, sorted(ks)
    k = ks[main[0]]
    b = k["body"]
    assert k["spill"] == 0 and "scratch_" not in b
    assert k["vgpr"] <= 256  # 2 waves per SIMD
    assert k["lds"] == 131072
    assert len(re.findall(r"s_waitcnt vmcnt\(0\)", b)) == 1  # only the post-loop drain
    assert len(re.findall(r"s_waitcnt vmcnt\(10\)", b)) >= 8  # counted waits in the loop
    assert len(re.findall(r"v_mfma_f32_16x16x32_bf16", b)) == 128  # 2 K-tiles unrolled
    assert len(re.findall(r"buffer_load_dwordx4 .* lds", b)) >= 16
    assert len(re.findall(r"ds_read_b64_tr_b16", b)) >= 32  # NN B operand, no transposed copy


def test_f32_kernel_no_spill(tmp_path):
    ks = _kernels("gemm_f32_256.hip", tmp_path, experiments=True)
    assert ks
    for name, k in ks.items():
        assert k["spill"] == 0 and "scratch_" not in k["body"], name
        assert k["vgpr"] <= 256, name
        # two K-tiles unrolled (256 MFMAs each); f32_256p's branch-free loop runs one per trip
        want = 256 if "gemm_f32_256p" in name else 512
        assert len(re.findall(r"v_mfma_f32_16x16x4_f32", k["body"])) == want, name


def test_bf16_two_quadrant_schedule(tmp_path):
    """SCHED 3: 32 MFMAs per compute slot, 4 barriers per K-tile, vmcnt(6) waits."""
    ks = _kernels("gemm_mfma256.hip", tmp_path)
    name = [k for k in ks if "gemm256_nn" in k and "ILi2ELi3ELb0ELi0E" in k]
    assert name, sorted(ks)
    k = ks[name[0]]
    b = k["body"]
    assert k["spill"] == 0 and k["vgpr"] <= 256
    assert len(re.findall(r"s_waitcnt vmcnt\(0\)", b)) == 1
    assert len(re.findall(r"s_waitcnt vmcnt\(6\)", b)) >= 4
    assert len(re.findall(r"v_mfma_f32_16x16x32_bf16", b)) == 128


def test_w4_kernel_agpr_accumulators_and_counted_waits(tmp_path):
    """gemm_w4.hip: 256 AGPR accumulators, no spills, 128 KiB LDS + the fused last
    K-tile's epilogue buffers (1 workgroup/CU),
    counted vmcnt(16) waits at the two barriers of each K-tile and one vmcnt(0) drain."""
    ks = _kernels("gemm_w4.hip", tmp_path)
    for dt, mfma in (("ILi2E", "v_mfma_f32_16x16x32_bf16"), ("ILi1E", "v_mfma_f32_16x16x32_f16")):
        name = [k for k in ks if "gemm_w4_nn" in k and dt in k and "Lb1ELb0EE" in k]  # not signalled
        assert name, sorted(ks)
        k = ks[name[0]]
        b = k["body"]
        assert k["spill"] == 0 and k["lds"] == 2 * 65536 + 4 * 4224  # + fused epilogue buffers
        assert re.search(r"v_mfma_f32_16x16x32_\w+ a\[", b)  # accumulators live in AGPRs
        assert k["vgpr"] <= 256
        assert "global_atomic" in b  # the fused split-K meeting point is compiled in
        # the K-loop (the backward branch over 2 K-tiles' 256 MFMAs) drains nothing: its
        # waits are the counted vmcnt(16) ones; the drains sit outside it (before the
        # separate epilogue and at the fused last K-tile's exit). Found by its back edge,
        # not by block order, which the compiler is free to change.
        loops = _loops(b, min_mfma=256)
        assert len(loops) == 1, [n for n, _ in loops]
        body = loops[0][1]
        assert not re.findall(r"s_waitcnt vmcnt\(0\)", body)
        assert len(re.findall(r"s_waitcnt vmcnt\(16\) lgkmcnt\(0\)", body)) >= 4
        assert len(re.findall(r"s_waitcnt vmcnt\(0\)", b)) >= 2
        # loop body: 2 K-tiles x 8 blocks x 16 MFMAs, one odd tail K-tile, the fused last K-tile
        assert len(re.findall(mfma, b)) == 4 * 128
        assert len(re.findall(r"buffer_load_dwordx4 .* lds", b)) >= 3 * 16


def test_w4_signalled_variant_publishes_write_through(tmp_path):
    """gemm_w4.hip SIG (completion signals, parallel/overlap.py): every C store is a
    write-through (sc1) buffer store — none of the plain / non-temporal global
    stores of the shipping epilogue — the K-loop is the plain kernel's, and each
    workgroup's signal is one returning agent atomic add behind an explicit
    vmcnt(0) drain and a barrier, then a system-scope flag store."""
    ks = _kernels("gemm_w4.hip", tmp_path)
    for dt in ("ILi2E", "ILi1E"):
        sig = [k for k in ks if "gemm_w4_nn" in k and dt in k and "Lb1ELb1EE" in k]
        plain = [k for k in ks if "gemm_w4_nn" in k and dt in k and "Lb1ELb0EE" in k]
        assert sig and plain, sorted(ks)
        b, p = ks[sig[0]]["body"], ks[plain[0]]["body"]
        assert ks[sig[0]]["spill"] == 0 and ks[sig[0]]["vgpr"] <= 256
        assert not re.findall(r"global_store_dwordx4", b)  # C leaves only as sc1 buffer stores
        assert len(re.findall(r"buffer_store_dwordx4 .* sc1", b)) >= 2 * 64
        assert len(re.findall(r"s_waitcnt vmcnt\(16\) lgkmcnt\(0\)", b)) == \
            len(re.findall(r"s_waitcnt vmcnt\(16\) lgkmcnt\(0\)", p))
        # the signal's own drain (asm, invisible to the compiler) on top of the plain kernel's
        drain = r";;#ASMSTART\s+s_waitcnt vmcnt\(0\)\s+;;#ASMEND"
        assert len(re.findall(drain, b)) == len(re.findall(drain, p)) + 1
        i_flag = b.find("sc0 sc1")  # the system-scope host-flag store
        i_add = b.rfind("global_atomic_add", 0, i_flag)  # the slot counter add it follows
        assert 0 <= i_add < i_flag and " sc0" in b[i_add:b.find("\n", i_add)]  # returning add
        assert b[i_add:i_flag].count("s_waitcnt vmcnt(0)") >= 1  # the flag waits for the add


def test_default_build_has_no_experiment_kernels(tmp_path):
    """The shipping library instantiates only the shipping schedules."""
    ks = _kernels("gemm_mfma256.hip", tmp_path)
    assert ks and all("ELi3ELb0ELi0EE" in k for k in ks), sorted(ks)  # SCHED 3 only
    (tmp_path / "fp8").mkdir()
    ks = _kernels("gemm_fp8.hip", tmp_path / "fp8")
    assert ks and all("gemm_fp8_w4ILi0ELi0E" in k or "gemm_fp8_w4s" in k or "gemm_fp8_sk" in k
                      for k in ks), sorted(ks)


def test_fp8_stream_k_kernel(tmp_path):
    """gemm_fp8_sk (stream-K over a tile range): no scratch (per-lane values are
    formed per segment, share arithmetic stays scalar), AGPR accumulators, one
    workgroup per CU, and its K-loop is W4's (counted vmcnt(16) waits at both
    barriers of each K-tile, no drain inside)."""
    ks = _kernels("gemm_fp8.hip", tmp_path)
    name = [k for k in ks if "gemm_fp8_sk" in k]
    assert name, sorted(ks)
    k = ks[name[0]]
    b = k["body"]
    assert k["spill"] == 0 and "scratch_" not in b
    assert k["lds"] == 2 * 65536
    assert re.search(r"v_mfma_f32_16x16x128_f8f6f4 a\[", b)
    loops = _loops(b, min_mfma=128)
    inner = [t for _, t in loops if not re.findall(r"s_waitcnt vmcnt\(0\)", t)]
    assert inner, [n for n, _ in loops]  # the 2-K-tile loop body, drain-free
    assert len(re.findall(r"s_waitcnt vmcnt\(16\) lgkmcnt\(0\)", inner[0])) >= 4


@pytest.mark.parametrize("src,pat,dts,zero_per_kt", [
    ("gemm_w4.hip", "gemm_w4s", ("ILi2E", "ILi1E"), 64),   # bf16 / fp16: C = 0 on ks = 0 only
    ("gemm_fp8.hip", "gemm_fp8_w4s", ("",), 64),           # fp8: one MFMA per accumulator
])
def test_streaming_kernels_structure(tmp_path, src, pat, dts, zero_per_kt):
    """W4S / fp8 W4S: no scratch, AGPR accumulators, the boundary's counted
    waits vmcnt(48) (32 epilogue stores younger than the awaited DMAs), each
    tile started by C = 0 MFMAs (no zeroing), 32 placeholder LDS-DMA loads,
    and exactly one vmcnt(0) drain (at exit): no compiler-inserted wait may
    drain the stream."""
    ks = _kernels(src, tmp_path)
    for dt in dts:
        name = [k for k in ks if pat + dt in k]
        assert name, sorted(ks)
        k = ks[name[0]]
        b = k["body"]
        assert k["spill"] == 0 and "scratch_" not in b, name
        assert k["lds"] == 2 * 65536 + 4 * 4224
        assert re.search(r"v_mfma_f32_16x16x\d+_\w+ a\[", b)
        assert len(re.findall(r"s_waitcnt vmcnt\(48\) lgkmcnt\(0\)", b)) == 3
        assert len(re.findall(r"v_mfma_f32_16x16x\d+_\w+ a\[\d+:\d+\], v\[\d+:\d+\], v\[\d+:\d+\], 0$",
                              b, re.M)) == zero_per_kt
        assert len(re.findall(r"s_waitcnt vmcnt\(0\)", b)) == 1
        assert len(re.findall(r"global_store_dwordx4", b)) == 32


EPI4 = 4 * 16 * (4 * 32 + 8)  # the fused last K-tile's per-wave epilogue buffers (epi_buf<4>)


@pytest.mark.parametrize("cfg,lds,waitn,mfma_per_kt,pieces", [
    ("Li128ELi128ELi4ELi1E", 4 * 32768 + EPI4, 16, 32, 8),    # T128: 4-stage ring
    ("Li256ELi128ELi3ELi1E", 3 * 49152 + EPI4, 12, 64, 12),   # T256x128: 3-stage ring
])
def test_tile_family_pipelined(tmp_path, cfg, lds, waitn, mfma_per_kt, pieces):
    """gemm_tile.hip (1 workgroup / CU members): no spills, AGPR accumulators,
    one vmcnt(P*(NS-2))-counted barrier per K-tile, vmcnt(0) only at the exits
    (before the split-K / unfused epilogue and after the fused last K-tile), prologue
    + 3 unrolled K-tiles of DMA pieces, sc1 slots."""
    ks = _kernels("gemm_tile.hip", tmp_path)
    for dt, mfma in (("ILi2E", "v_mfma_f32_16x16x32_bf16"), ("ILi1E", "v_mfma_f32_16x16x32_f16")):
        name = [k for k in ks if "gemm_tile_nn" + dt in k and cfg in k and "Lb1E" in k]
        assert name, sorted(ks)
        k = ks[name[0]]
        b = k["body"]
        assert k["spill"] == 0 and k["lds"] == lds and k["vgpr"] <= 256
        assert re.search(r"v_mfma_f32_16x16x32_\w+ a\[", b)
        head = b[:b.find("global_atomic")]
        assert 1 <= len(re.findall(r"s_waitcnt vmcnt\(0\)", head)) <= 2  # unfused / split-K (+ fused exit)
        kloop = re.search(r"Inner Loop Header.*?s_cbranch_(?:scc1|vccnz) \.LBB", b, re.S).group(0)
        assert "vmcnt(0)" not in kloop and "v_mfma" in kloop  # the K-loop never drains
        assert len(re.findall(r"s_waitcnt vmcnt\(0\)", b[b.rfind("v_mfma"):])) >= 1  # the fused exit's drain
        assert len(re.findall(rf"s_waitcnt vmcnt\({waitn}\) lgkmcnt\(0\)", b)) == 3
        # 2 unrolled K-tiles + the odd tail + the fused last K-tile
        assert len(re.findall(mfma, b)) == 4 * mfma_per_kt
        stages = lds // (lds // {16: 4, 12: 3}[waitn])
        assert len(re.findall(r"buffer_load_dwordx4 .* lds", b)) == (stages + 3) * pieces
        assert len(re.findall(r"buffer_store_dwordx4 .* sc1", b)) == mfma_per_kt // 2  # slots


def test_t128x2_two_workgroups_per_cu(tmp_path):
    """The 2-stage T128 variant: 64 KiB LDS and <= 256 VGPR + AGPR per wave, so two
    256-thread workgroups fit on a CU; its loop waits vmcnt(0) at every K-tile top
    (+1: the barrier before the LDS-staged epilogue)."""
    ks = _kernels("gemm_tile.hip", tmp_path)
    name = [k for k in ks if "gemm_tile_nnILi2E" in k and "Li128ELi128ELi2ELi2E" in k]
    assert name, sorted(ks)
    k = ks[name[0]]
    assert k["spill"] == 0 and k["lds"] == 2 * 32768
    assert k["vgpr"] <= 128
    assert len(re.findall(r"s_waitcnt vmcnt\(0\) lgkmcnt\(0\)", k["body"])) == 4
