"""One gfx950 compile per (source, build flavour) per test process, shared by
the static assembly checks (test_kernel_asm.py, test_mfma_hazards.py)."""
import functools
import os
import shutil
import subprocess
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_distributed_matmul_benchmark_amd", "ops", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")


@functools.lru_cache(maxsize=None)
def gfx950_asm(src: str, experiments: bool = False) -> str:
    """The device assembly (.s text) of ``csrc/src`` (default build, or with the
    A/B experiment kernels)."""
    d = tempfile.mkdtemp(prefix="pdmb_asm_")
    try:
        defs = ["-DPDMB_EXPERIMENTS=1"] if experiments else []
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", *defs, "-c",
                        os.path.join(CSRC, src), "-o", os.path.join(d, "k.o"), "-save-temps"],
                       cwd=d, check=True, capture_output=True, timeout=900)
        s = next(f for f in os.listdir(d) if "gfx950" in f and f.endswith(".s"))
        with open(os.path.join(d, s)) as fh:
            return fh.read()
    finally:
        shutil.rmtree(d, ignore_errors=True)
