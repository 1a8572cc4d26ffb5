#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` result (rocpd SQLite ``*.db`` or
``*_kernel_stats.csv``) into a short markdown table: per-kernel calls, total
and mean time, share of GPU time, plus grid / VGPR / LDS of each kernel.

    python scripts/rocprof_summary.py gpurun_out/rocprof/bench_results.db > profiles/x.md
"""
from __future__ import annotations

import csv
import re
import sqlite3
import sys


def short(name: str, width: int = 90) -> str:
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration), max(grid_x), max(workgroup_x), max(vgpr_count), "
                     "max(accum_vgpr_count), max(sgpr_count), max(lds_size) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    out = ["| kernel | calls | total ms | mean µs | min µs | max µs | % GPU | grid | wg | vgpr | agpr | sgpr | lds B |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{short(r[0])}` | {r[1]} | {r[2] / 1e6:.3f} | {r[3] / 1e3:.1f} | "
                   f"{r[4] / 1e3:.1f} | {r[5] / 1e3:.1f} | {100 * r[2] / total:.1f} | {r[6]} | "
                   f"{r[7]} | {r[8]} | {r[9]} | {r[10]} | {r[11]} |")
    return out


def from_csv(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    out = ["| kernel | calls | total ms | mean µs | % GPU |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    return out


def main(argv):
    for p in argv[1:]:
        print(f"### {p}\n")
        print("\n".join(from_db(p) if p.endswith(".db") else from_csv(p)))
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
