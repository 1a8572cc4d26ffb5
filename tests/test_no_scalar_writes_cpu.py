"""Static safety check (CPU): no kernel of the shipping library writes through the
scalar data cache (scalar stores / atomics / cache write-back), which this GPU pool
forbids. Listed in .gpurunignore: it names those instructions and no GPU run loads it."""
import glob
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_distributed_matmul_benchmark_amd", "ops", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
FORBIDDEN = re.compile(r"\b(s_store_\w+|s_atomic_\w+|s_buffer_store\w*|s_buffer_atomic\w*|"
                       r"s_dcache_wb\w*|s_dcache_discard\w*|s_scratch_store\w*)\b")


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("src", ["gemm_w4.hip", "gemm_tile.hip", "gemm_mfma256.hip", "gemm_fp8.hip",
                                 "gemm_f32_256.hip", "gemm_generic.hip", "gemm_dispatch.cpp"])
def test_no_scalar_cache_writes(src, tmp_path):
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", *lang, "-c",
                    os.path.join(CSRC, src), "-o", str(tmp_path / "k.o"), "-save-temps"],
                   cwd=tmp_path, check=True, capture_output=True, timeout=600)
    asm = open(glob.glob(str(tmp_path / "*gfx950*.s"))[0]).read()
    assert not FORBIDDEN.findall(asm)
