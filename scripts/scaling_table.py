#!/usr/bin/env python3
"""Merge ``--json`` records (or bench.py JSON lines) from 1/2/4/8-GPU runs into
the BASELINE scaling table: node TFLOPS per (mode, N, dtype, world size) and
scaling efficiency = node TFLOPS / (ws × the 1-GPU node TFLOPS of the same
mode, size and dtype).

    python scripts/scaling_table.py results/*.jsonl [--size 16384] [--markdown]
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import defaultdict


def load(paths):
    recs = []
    for p in paths:
        with open(p) as f:
            for line in f:
                line = line.strip()
                if not line.startswith("{"):
                    continue
                r = json.loads(line)
                if "metric" in r and "value" in r:  # bench.py line
                    c = r.get("config", {})
                    n = c.get("seq_len")
                    r = {"mode": c.get("mode", "independent") + ("+overlap" if c.get("overlap") else ""),
                         "n": n, "dtype": r.get("dtype"), "world_size": r["n_gpus"],
                         "node_tflops": r["value"], "max_ms": r["ms_per_step"]}
                elif "error" in r:
                    continue
                else:
                    if r.get("overlap"):
                        r = dict(r, mode=r["mode"] + "+overlap")
                    if r.get("backend", "native") != "native":
                        r = dict(r, mode=f"{r['mode']} [{r['backend']}]")
                recs.append(r)
    return recs


def table(recs, size=None):
    best = {}
    for r in recs:
        if size and r.get("n") != size:
            continue
        key = (r["mode"], r.get("n"), r.get("dtype"), int(r["world_size"]))
        if key not in best or r["node_tflops"] > best[key]["node_tflops"]:
            best[key] = r
    groups = defaultdict(dict)
    for (mode, n, dt, ws), r in best.items():
        groups[(mode, n, dt)][ws] = r
    rows = []
    for (mode, n, dt), byws in sorted(groups.items(), key=lambda kv: tuple(map(str, kv[0]))):
        one = byws.get(1, {}).get("node_tflops")
        for ws in sorted(byws):
            t = byws[ws]["node_tflops"]
            eff = 100.0 * t / (ws * one) if one else None
            rows.append((mode, n, dt, ws, t, eff))
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("files", nargs="+")
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--markdown", action="store_true")
    a = ap.parse_args(argv)
    rows = table(load(a.files), a.size)
    if a.markdown:
        print("| mode | N | dtype | GPUs | node TFLOPS | scaling eff. vs 1 GPU |")
        print("|---|---|---|---|---|---|")
        for m, n, dt, ws, t, e in rows:
            print(f"| {m} | {n} | {dt} | {ws} | {t:.1f} | {'' if e is None else f'{e:.1f}%'} |")
    else:
        print(f"{'mode':24s} {'N':>6s} {'dtype':>9s} {'GPUs':>4s} {'node TFLOPS':>12s} {'eff':>7s}")
        for m, n, dt, ws, t, e in rows:
            print(f"{m:24s} {n!s:>6s} {dt!s:>9s} {ws:4d} {t:12.1f} "
                  f"{'   n/a' if e is None else f'{e:6.1f}%'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
