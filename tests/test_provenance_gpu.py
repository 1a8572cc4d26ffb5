"""Provenance: under rocprofv3 --kernel-trace, the timed GEMMs of bench.py are this
package's gfx950 kernels — no rocBLAS / hipBLASLt (``Cijk_*``) kernel runs."""
import csv
import glob
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("rocprofv3") is None, reason="rocprofv3 not installed")
def test_bench_runs_only_native_gemm_kernels(tmp_path):
    out = tmp_path / "prof"
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", str(out),
                        "-o", "run", "--", sys.executable, "bench.py", "--size", "4096",
                        "--steps", "5", "--warmup", "1"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    files = glob.glob(str(out / "**" / "*kernel_trace.csv"), recursive=True)
    assert files, "no kernel trace written"
    names = [row["Kernel_Name"] for f in files for row in csv.DictReader(open(f))]
    gemms = [n for n in names if "gemm" in n.lower() or n.startswith("Cijk")]
    assert len([n for n in gemms if "pdmb::" in n]) >= 6  # warmup + 5 timed steps
    assert not [n for n in names if n.startswith("Cijk") or "rocblas" in n.lower()], set(names)
