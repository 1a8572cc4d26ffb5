"""Rank-0 console report (reference-compatible lines) + machine-readable records.

The reference's only output is rank-0 ``print`` lines, and
``backup/compare_benchmarks.py:19-26`` scrapes them for ``16384x16384``,
``Results for``, ``Average time``, ``TFLOPS`` and ``overhead``. Those
substrings are kept verbatim so existing scrapers keep working. In
addition every (script, mode, N, dtype, ws) result becomes one JSON record
(``--json``) with unambiguous fields, which the sweep tool merges into the
1/2/4/8-GPU scaling table.
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time
from typing import Any, Dict, List, Optional

import torch

from .metrics import dtype_name


class Reporter:
    def __init__(self, is_main: bool = True, stream=None, json_path: Optional[str] = None):
        self.is_main = is_main
        self.stream = stream or sys.stdout
        self.json_path = json_path
        self.records: List[Dict[str, Any]] = []

    def line(self, text: str = "") -> None:
        if self.is_main:
            print(text, file=self.stream, flush=True)

    def rule(self, width: int = 60) -> None:
        self.line("=" * width)

    def record(self, rec: Dict[str, Any]) -> None:
        if not self.is_main:
            return
        rec = dict(rec)
        rec.setdefault("timestamp", time.time())
        self.records.append(rec)
        if self.json_path:
            d = os.path.dirname(os.path.abspath(self.json_path))
            os.makedirs(d, exist_ok=True)
            with open(self.json_path, "a") as f:
                f.write(json.dumps(rec, default=_jsonable) + "\n")


def _jsonable(o):
    if isinstance(o, torch.dtype):
        return dtype_name(o)
    if isinstance(o, torch.device):
        return str(o)
    return str(o)


def device_banner(rep: Reporter, device: torch.device) -> None:
    """Environment banner (matmul_scaling_benchmark.py:376-386), ROCm-aware:
    prints the HIP version instead of ``torch.version.cuda`` (None on ROCm)
    and reports CUs (not "SMs") with the gfx ISA."""
    rep.line(f"PyTorch version: {torch.__version__}")
    gpu = torch.cuda.is_available()
    rep.line(f"CUDA available: {gpu}")
    if gpu:
        hip = getattr(torch.version, "hip", None)
        if hip:
            rep.line(f"HIP (ROCm) version: {hip}")
        else:
            rep.line(f"CUDA version: {torch.version.cuda}")
        n = torch.cuda.device_count()
        rep.line(f"Number of CUDA devices: {n}")
        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            rep.line(f"  GPU {i}: {torch.cuda.get_device_name(i)}")
            rep.line(f"    Memory: {p.total_memory / (1024 ** 3):.2f} GB")
            arch = getattr(p, "gcnArchName", "")
            rep.line(f"    SMs: {p.multi_processor_count}" + (f" (CUs, {arch})" if arch else ""))
    if device.type == "cpu":
        rep.line(f"Device: CPU ({platform.processor() or platform.machine()}, "
                 f"{torch.get_num_threads()} threads)")


def fmt_opt(v: Optional[float], spec: str = ".1f", suffix: str = "") -> str:
    return "n/a" if v is None else f"{v:{spec}}{suffix}"
