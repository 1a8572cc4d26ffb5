"""Static hazard screen of the generated gfx950 code around the inline-asm MFMAs
(CPU only: hipcc cross-compiles).

The hot kernels issue their MFMAs as inline asm (fixed AGPR accumulators, exact
issue order), so hipcc's hazard recognizer does not know those instructions are
MFMAs: a register copy the compiler places right before one (a VALU write of a
VGPR / AGPR that the MFMA then reads as SrcA/B/C) gets no wait states, and the
MFMA reads the stale value. That is how the fp32 two-stage tile kernel returned
wrong results at odd K / 32 when an unrelated epilogue change raised its
register pressure (``v_mov_b64 v[0:1], ...`` one instruction before
``v_mfma ... v0 ...``; scripts/race_screen.py found it on the GPU). This test
finds the pattern in the assembly of every kernel of the default build, so the
next such codegen change fails here, before any GPU run.

Rule checked (gfx950, as for gfx940: a VALU write followed by an MFMA read of
the same register needs 2 wait states; ``s_nop N`` counts N + 1), over the
linear instruction stream, across block boundaries. One pattern is exempt: a
``v_accvgpr_write aR, vX`` whose ``vX`` was read from ``aR`` itself with nothing
writing either in between (the compiler parking an accumulator in a VGPR and
putting it back): the MFMA reads the same value either way.
"""
import os
import re
import shutil

import pytest
from asm_cache import gfx950_asm

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_distributed_matmul_benchmark_amd", "ops", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")

SOURCES = ["gemm_w4.hip", "gemm_fp8.hip", "gemm_tile.hip", "gemm_f32_tile.hip", "gemm_f32_w4.hip",
           "gemm_f32_256.hip", "gemm_mfma256.hip"]
MEM = ("ds_", "buffer_", "global_", "flat_", "scratch_")
NEED = 2  # VALU write -> MFMA read wait states


def _regs(tok):
    tok = tok.strip()
    m = re.match(r"([av])\[(\d+):(\d+)\]$", tok)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([av])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def _instructions(body):
    out = []
    for line in body.splitlines():
        line = line.split(";")[0].strip()
        if line and not line.startswith(".") and not line.endswith(":"):
            out.append(line)
    return out


def _dst(ins):
    op = ins.split()[0]
    return _regs(ins[len(op):].split(",")[0])


def _parked(ins, j):
    """ins[j] = v_accvgpr_write aR, vX, with vX read from aR earlier and neither
    register written in between."""
    m = re.match(r"v_accvgpr_write_b32 a(\d+), v(\d+)$", ins[j])
    if not m:
        return False
    a, v = ("a", int(m.group(1))), ("v", int(m.group(2)))
    for k in range(j - 1, max(-1, j - 2000), -1):
        if re.match(rf"v_accvgpr_read_b32 v{v[1]}, a{a[1]}$", ins[k]):
            return True
        op = ins[k].split()[0]
        if op.startswith("s_"):
            continue
        if (a in _dst(ins[k]) or v in _dst(ins[k])) and not op.startswith(("buffer_store", "global_store")):
            return False
    return False


def hazards(body):
    ins = _instructions(body)
    bad = []
    for i, line in enumerate(ins):
        op = line.split()[0]
        if not op.startswith("v_mfma"):
            continue
        srcs = set().union(*(_regs(t) for t in line[len(op):].split(",")[1:4]))
        states = 0
        for j in range(i - 1, max(-1, i - 8), -1):
            pj = ins[j].split()[0]
            if pj == "s_nop":
                states += int(ins[j].split()[1], 0) + 1
            else:
                if (pj.startswith("v_") and not pj.startswith("v_mfma") and not pj.startswith(MEM)
                        and _dst(ins[j]) & srcs and not _parked(ins, j)):
                    bad.append((ins[j], line, states))
                states += 1
            if states >= NEED:
                break
    return bad


def _kernels(text):
    for m in re.finditer(r"^([A-Za-z_][\w.$]*):\s*;\s*@", text, re.M):
        yield m.group(1), text[m.end():text.find(".Lfunc_end", m.end())]


def test_detects_the_fp32_odd_tail_pattern():
    """The exact sequence the broken fp32 two-stage build had."""
    body = "\n".join(["\tv_mfma_f32_16x16x4_f32 a[20:23], v37, v110, a[20:23]",
                      "\tv_mov_b64_e32 v[0:1], v[14:15]", "\tv_mov_b64_e32 v[2:3], v[16:17]",
                      "\tv_mfma_f32_16x16x4_f32 a[8:11], v34, v0, a[8:11]"])
    assert len(hazards(body)) == 1
    ok = body.replace("\tv_mov_b64_e32 v[2:3]", "\ts_nop 1\n\tv_mov_b64_e32 v[2:3]")
    assert hazards(ok) == []  # v0 is written 3 states before the read


def test_parked_accumulator_is_exempt():
    body = "\n".join(["\tv_accvgpr_read_b32 v90, a204", "\tv_add_f32 v1, v2, v3",
                      "\tv_accvgpr_write_b32 a204, v90",
                      "\tv_mfma_f32_16x16x32_bf16 a[204:207], v[174:177], v[134:137], a[204:207]"])
    assert hazards(body) == []
    assert len(hazards(body.replace("v_add_f32 v1", "v_add_f32 v90"))) == 1


@pytest.mark.parametrize("src", SOURCES)
def test_no_valu_write_right_before_an_mfma_read(src):
    found = {name: h for name, body in _kernels(gfx950_asm(src)) if (h := hazards(body))}
    assert not found, {k[:90]: v[:3] for k, v in found.items()}


# The other direction (round 6): an MFMA's result read by a VALU instruction
# (v_accvgpr_read / v_accvgpr_mov of the accumulator, or any VALU source) too
# soon after the MFMA that writes it. The streamed exact-fp32 kernel's epilogue
# regroup first had hipcc copy an accumulator tuple ONE instruction after the
# MFMA that wrote it (profiles/r8lq_fp32_lean_stream.md); every accumulator is
# now an operand of the s_nop padding instead. The bound checked is 8 wait
# states: the closest such read in the shipping build is the fp8 tile
# family's epilogue at 8 (16x16x128 f8f6f4), 13 for its bf16 / fp16 members,
# >= 25 everywhere else, and the tile family is exact on small integers on the
# GPU (tests/test_fp8_gpu.py::test_fp8_tile_family_exact, test_gemm_gpu.py).
NEED_RD = 8


def _srcs(ins):
    op = ins.split()[0]
    return set().union(*(_regs(t) for t in ins[len(op):].split(",")[1:]))


def read_hazards(body):
    ins = _instructions(body)
    bad = []
    for i, line in enumerate(ins):
        op = line.split()[0]
        if not op.startswith("v_mfma"):
            continue
        dst = _dst(line)
        states = 0
        for j in range(i + 1, min(len(ins), i + 40)):
            pj = ins[j].split()[0]
            if pj in ("s_branch", "s_setpc_b64", "s_endpgm"):
                break  # no fall-through: what follows is another block's code
            if pj == "s_nop":
                states += int(ins[j].split()[1], 0) + 1
            else:
                if pj.startswith("v_") and not pj.startswith("v_mfma") and _srcs(ins[j]) & dst:
                    bad.append((line, ins[j], states))
                    break
                if pj.startswith("v_mfma") and _dst(ins[j]) & dst:
                    break  # rewritten by the next MFMA (same-pipe ordering)
                dst = dst - _dst(ins[j])  # overwritten: later reads see that value
                if not dst:
                    break
                states += 1
            if states >= NEED_RD:
                break
    return bad


def test_detects_a_copy_right_after_the_mfma():
    body = "\n".join(["\tv_mfma_f32_16x16x4_f32 a[240:243], v105, v69, a[240:243]", "\ts_nop 0",
                      "\tv_accvgpr_read_b32 v88, a240"])
    assert len(read_hazards(body)) == 1
    ok = body.replace("\ts_nop 0", "\ts_nop 15")
    assert read_hazards(ok) == []
    # not reached by fall-through, or the register rewritten first: no hazard
    assert read_hazards(body.replace("\ts_nop 0", "\ts_branch .LBB0_9\n.LBB0_8:")) == []
    assert read_hazards(body.replace("\ts_nop 0", "\tv_accvgpr_write_b32 a240, 0")) == []


@pytest.mark.parametrize("src", SOURCES)
def test_no_valu_read_right_after_an_mfma_write(src):
    found = {name: h for name, body in _kernels(gfx950_asm(src)) if (h := read_hazards(body))}
    assert not found, {k[:90]: v[:3] for k, v in found.items()}
