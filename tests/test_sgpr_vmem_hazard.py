"""Static screen for the VALU-writes-SGPR -> VMEM-reads-SGPR hazard around the
inline-asm LDS-DMA pieces (CPU only: hipcc cross-compiles).

On gfx9-family chips (gfx950 included) a VMEM instruction that reads an SGPR
(descriptor or soffset) must come at least 5 wait states after a VALU
instruction that wrote it (v_readlane / v_readfirstlane, a v_cmp with an SGPR
result, a carry-out). hipcc pads its own loads (``s_nop 3`` after
``v_readfirstlane`` + ``s_mul``, checked below on a probe), but the kernels issue
their LDS-DMA as inline asm, whose operand reads it does not see. Round 6 found
W4S and fp8 W4S restoring a spilled soffset with ``v_readlane`` 2 wait states
before a DMA piece of a tile's first K-tiles (4 sites in bf16 W4S, 1 in fp8
W4S); those K-tiles now issue their pieces through ``dma16_at_pad`` (common.h).
This test scans every default-build kernel for the pattern.
"""
import re

import pytest
from asm_cache import HIPCC, gfx950_asm
from test_mfma_hazards import _instructions, _kernels

pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")

SOURCES = ["gemm_w4.hip", "gemm_fp8.hip", "gemm_tile.hip", "gemm_f32_tile.hip", "gemm_f32_w4.hip",
           "gemm_f32_256.hip", "gemm_mfma256.hip"]
NEED = 5
VMEM = ("buffer_", "global_", "flat_", "scratch_")


def _sregs(tok):
    tok = tok.strip()
    m = re.match(r"s\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _valu_sgpr_dst(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return set()
    ops = [t for t in re.split(r"[ ,]+", ins[len(op):].strip()) if t]
    if op.startswith(("v_readfirstlane", "v_readlane")) or (op.startswith("v_cmp") and not op.startswith("v_cmpx")):
        return _sregs(ops[0]) if ops else set()
    if op.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_addc", "v_subb", "v_mad_u64", "v_mad_i64",
                      "v_div_scale")) and len(ops) > 1:
        return _sregs(ops[1])
    return set()


def hazards(body):
    ins = _instructions(body)
    bad = []
    for i, line in enumerate(ins):
        op = line.split()[0]
        if not op.startswith(VMEM):
            continue
        srcs = set().union(*(_sregs(t) for t in re.split(r"[ ,]+", line[len(op):]) if t))
        if not srcs:
            continue
        states = 0
        for j in range(i - 1, max(-1, i - 12), -1):
            pj = ins[j].split()[0]
            if pj in ("s_branch", "s_setpc_b64", "s_endpgm") or pj.startswith("s_cbranch"):
                break  # another block's code (conservative)
            if pj == "s_nop":
                states += int(ins[j].split()[1], 0) + 1
            else:
                if _valu_sgpr_dst(ins[j]) & srcs:
                    bad.append((ins[j], line, states))
                    break
                states += 1
            if states >= NEED:
                break
    return bad


def test_detects_the_w4s_pattern():
    body = "\n".join(["\tv_readlane_b32 s21, v254, 23", "\ts_add_u32 m0, s98, 0x12000", "\ts_nop 0",
                      "\tbuffer_load_dwordx4 v210, s[36:39], s21 offen lds"])
    assert len(hazards(body)) == 1
    assert hazards(body.replace("\ts_nop 0", "\ts_nop 3")) == []


def test_hipcc_pads_its_own_loads_this_way():
    """The rule this test enforces is hipcc's own: a v_readfirstlane feeding a
    buffer load's soffset gets 5 wait states."""
    import os
    import subprocess
    import tempfile
    src = r'''
#include <hip/hip_runtime.h>
__global__ void k(const float* p, float* out, int x) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 1 << 30, 0x00020000);
  int lane = __builtin_amdgcn_mbcnt_lo(~0u, 0u);
  int voff = lane * 4;
  asm volatile("" : "+v"(voff));
  __builtin_amdgcn_sched_barrier(0);
  int v = __builtin_amdgcn_readfirstlane(lane * x);
  out[lane] = __builtin_amdgcn_raw_buffer_load_b32(r, voff, v, 0);
}
'''
    d = tempfile.mkdtemp(prefix="pdmb_hz_")
    with open(os.path.join(d, "t.hip"), "w") as f:
        f.write(src)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-c", "t.hip", "-o", "t.o", "-save-temps"], cwd=d,
                   check=True, capture_output=True, timeout=300)
    s = next(f for f in os.listdir(d) if "gfx950" in f and f.endswith(".s"))
    with open(os.path.join(d, s)) as fh:
        body = fh.read()
    assert "v_readfirstlane" in body and "buffer_load" in body
    assert hazards(body) == []  # hipcc kept >= 5 wait states


@pytest.mark.parametrize("src", SOURCES)
def test_no_valu_sgpr_write_right_before_a_vmem_read(src):
    found = {name: h for name, body in _kernels(gfx950_asm(src)) if (h := hazards(body))}
    assert not found, {k[:90]: v[:3] for k, v in found.items()}
