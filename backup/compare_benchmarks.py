#!/usr/bin/env python3
"""Run the four reference comparison tests and print their 16k result lines.

Reference: backup/compare_benchmarks.py:10-63 — runs
``run_benchmark.sh 2`` (independent), ``run_distributed_benchmark.sh 2
data_parallel``, ``run_overlap_benchmark.sh 2 no_overlap`` and ``… overlap``
through ``shell=True`` from the cwd (which works from no directory, SURVEY
Q14), ignores exit codes and scrapes stdout for lines after "16384x16384".

Here the launchers are resolved relative to this file, run without a shell,
their exit codes are checked, and the scraped lines are the same substrings
(``Results for``, ``Average time``, ``TFLOPS``, ``overhead``). ``--gpus``,
``--dtype``, ``--size`` and ``--extra`` (flags passed through to the
scripts, e.g. ``--extra "--sizes 4096 --iterations 5"``) are opt-in.
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KEYS = ("Results for", "Average time", "Total time", "TFLOPS", "overhead")


def run_benchmark(script: str, gpus: int, mode: str, dtype: str = "bfloat16",
                  size: int = 16384, extra=()) -> tuple:
    """Run one launcher; returns (returncode, stdout, scraped lines)."""
    path = os.path.join(ROOT if script == "run_benchmark.sh" else HERE, script)
    argv = ["bash", path, str(gpus)] + ([mode] if mode else []) + [dtype] + list(extra)
    print(f"\n{'=' * 70}\nRunning: {' '.join(shlex.quote(a) for a in argv)}\n{'=' * 70}", flush=True)
    r = subprocess.run(argv, capture_output=True, text=True)
    lines = r.stdout.split("\n")
    picked = []
    tag = f"Results for {size}x{size}"
    for i, line in enumerate(lines):
        if tag in line:
            for j in range(i, min(i + 18, len(lines))):
                if any(k in lines[j] for k in KEYS):
                    picked.append(lines[j])
    for p in picked:
        print(p)
    if r.returncode != 0:
        print(f"  FAILED (exit {r.returncode}):\n{r.stderr[-2000:]}", flush=True)
    return r.returncode, r.stdout, picked


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=2)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--size", type=int, default=16384, help="size whose results are scraped")
    ap.add_argument("--extra", default="", help="flags passed through to every benchmark script")
    a = ap.parse_args(argv)
    extra = shlex.split(a.extra)
    print("\n" + "=" * 80 + "\nCOMPREHENSIVE BENCHMARK COMPARISON\n" + "=" * 80)
    tests = [
        ("TEST 1: Original benchmark - Independent (no communication)", "run_benchmark.sh", ""),
        ("TEST 2: Distributed - Data Parallel (with allreduce)", "run_distributed_benchmark.sh",
         "data_parallel"),
        ("TEST 3: Overlap Benchmark - No Overlap", "run_overlap_benchmark.sh", "no_overlap"),
        ("TEST 4: Overlap Benchmark - With Overlap", "run_overlap_benchmark.sh", "overlap"),
    ]
    failures = 0
    for title, script, mode in tests:
        print(f"\n### {title}")
        rc, _, _ = run_benchmark(script, a.gpus, mode, a.dtype, a.size, extra)
        failures += rc != 0
    print("\n" + "=" * 80 + "\nSUMMARY\n" + "=" * 80)
    print("""
    Key Metrics to Compare:
    1. Independent (no communication) = baseline maximum throughput
    2. Data Parallel (with allreduce) = realistic distributed training
    3. No Overlap = sequential compute then communicate
    4. With Overlap = overlapped compute and communicate (event-ordered ring)
    """)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
