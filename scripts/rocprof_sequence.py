#!/usr/bin/env python3
"""Kernel launches of a rocprofv3 ``--kernel-trace`` database in start order:
short name, duration and the gap since the previous kernel ended (µs). Reads
the same rocpd ``kernels`` view as rocprof_summary.py.

    python scripts/rocprof_sequence.py gpurun_out/x/rocprof/run_results.db [--grep pdmb] > seq.txt
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grep", default="", help="keep kernels whose name matches this regex")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    prev = None
    for name, start, end in rows:
        if a.grep and not re.search(a.grep, name):
            continue
        short = re.sub(r"\s+", " ", name)
        short = short if len(short) <= 70 else short[:67] + "..."
        gap = (start - prev) / 1e3 if prev is not None else 0.0
        print(f"{(end - start) / 1e3:10.1f} us  gap {gap:9.1f}  {short}")
        prev = end


if __name__ == "__main__":
    main()
