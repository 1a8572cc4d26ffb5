"""GPU interconnect report (the reference only prints a hint to run
``nvidia-smi topo -m``, backup/matmul_overlap_benchmark.py:397-402).

On an MI355X node every GPU pair is one xGMI hop (7 links × ~153 GB/s per
GPU); ``rocm-smi --showtopotype`` / ``--showtopohops`` show it. The report is
best-effort: a missing tool or driver yields a one-line note, never an error.
"""
from __future__ import annotations

import shutil
import subprocess
from typing import List


def topology_lines(timeout: float = 20.0) -> List[str]:
    exe = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi"
                                       if shutil.os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if exe is None:
        return ["(rocm-smi not found: no interconnect report)"]
    try:
        r = subprocess.run([exe, "--showtopotype", "--showtopohops"], capture_output=True,
                           text=True, timeout=timeout)
    except Exception as e:  # pragma: no cover - environment dependent
        return [f"(rocm-smi failed: {e!r})"]
    lines = [l.rstrip() for l in r.stdout.splitlines() if l.strip() and not set(l.strip()) <= set("=")]
    if r.returncode != 0 or not lines:
        return [f"(rocm-smi --showtopotype returned {r.returncode}: no interconnect report)"]
    return lines
