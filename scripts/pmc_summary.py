#!/usr/bin/env python3
"""Per-kernel PMC summary of ``scripts/gpu_pmc.sh`` output (rocprofv3 csv passes):
median duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / time), MFMA
utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs × cycles)), L2 hit rate,
LDS bank conflicts and wave stall split. Markdown to stdout.

    python scripts/pmc_summary.py gpurun_out/pmc
    python scripts/pmc_summary.py gpurun_out/pmc --cycle w4s,x_w4s_snake,torch

``--cycle``: label every GEMM dispatch by its position in the launch order
instead of by kernel name (scripts/prof_gemm_arms.py issues its arms in one
fixed cycle, the torch arm last): arms that run the same kernel template with
another runtime argument (a tile order) are told apart.
"""
import collections
import csv
import os
import statistics
import sys


def short(k):
    if k.startswith(("Cijk", "Custom_Cijk")):  # hipBLASLt (tuned kernels carry a Custom_ prefix)
        return "hipBLASLt " + k.split("_MT")[1].split("_")[0] if "_MT" in k else k[:40]
    return k.replace("void ", "").split("(")[0]


def main(d, cycle=None):
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        seen = set()
        rows = [r for r in csv.DictReader(open(f))
                if "distribution" not in r["Kernel_Name"] and "fillBuffer" not in r["Kernel_Name"]]
        if cycle:  # only the GEMMs take part in the cycle (fp8 runs also launch quantize kernels)
            rows = [r for r in rows if "pdmb::" in r["Kernel_Name"] or "Cijk" in r["Kernel_Name"]]
        order = {did: i for i, did in enumerate(sorted({int(r["Dispatch_Id"]) for r in rows}))}
        for r in rows:
            k = r["Kernel_Name"]
            if cycle:
                k = cycle[order[int(r["Dispatch_Id"])] % len(cycle)]
            cnt[short(k)][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (r["Dispatch_Id"], p)
            if key not in seen:
                seen.add(key)
                dur[short(k)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("| kernel | median µs | clock GHz | MFMA util | L2 hit | LDS bank confl. / LDS cycles | WAIT_ANY : WAIT_INST : ACTIVE |")
    print("|---|---|---|---|---|---|---|")
    for k, c in cnt.items():
        med = lambda n: statistics.median(c[n][1:] if len(c[n]) > 2 else c[n]) if c.get(n) else None  # noqa: E731
        t = statistics.median(dur[k][1:]) if len(dur[k]) > 2 else statistics.median(dur[k])
        g = med("GRBM_GUI_ACTIVE")
        clk = g / 8 / (t * 1e-6) / 1e9 if g else None
        mf = med("SQ_VALU_MFMA_BUSY_CYCLES")
        util = mf / 1024 / (g / 8) if (mf and g) else None
        hit, miss = med("TCC_HIT_sum"), med("TCC_MISS_sum")
        l2 = hit / (hit + miss) if hit is not None and miss else None
        bc, la = med("SQ_LDS_BANK_CONFLICT"), med("SQ_LDS_IDX_ACTIVE")
        wa, wi, ac = med("SQ_WAIT_ANY"), med("SQ_WAIT_INST_ANY"), med("SQ_ACTIVE_INST_ANY")
        f = lambda v, s: "n/a" if v is None else format(v, s)  # noqa: E731
        split = "n/a" if wa is None else f"{wa / 1e9:.2f} : {wi / 1e9:.2f} : {ac / 1e9:.2f} (×1e9)"
        print(f"| `{k}` | {t:.0f} | {f(clk, '.3f')} | {f(util, '.1%')} | {f(l2, '.1%')} | "
              f"{f(bc, '.3g')} / {f(la, '.3g')} | {split} |")
    if any(c.get("SQ_INSTS_MFMA") for c in cnt.values()):
        print()
        print("| kernel | MFMA insts | VALU / MFMA | SALU / MFMA | LDS / MFMA | SMEM / MFMA | VMEM / MFMA | BRANCH / MFMA |")
        print("|---|---|---|---|---|---|---|---|")
        for k, c in cnt.items():
            med = lambda n: statistics.median(c[n][1:] if len(c[n]) > 2 else c[n]) if c.get(n) else None  # noqa: E731
            mf = med("SQ_INSTS_MFMA")
            if not mf:
                continue
            r = lambda n: "n/a" if med(n) is None else f"{med(n) / mf:.4f}"  # noqa: E731
            print(f"| `{k}` | {mf:.4g} | {r('SQ_INSTS_VALU')} | {r('SQ_INSTS_SALU')} | {r('SQ_INSTS_LDS')} | "
                  f"{r('SQ_INSTS_SMEM')} | {r('SQ_INSTS_VMEM')} | {r('SQ_INSTS_BRANCH')} |")
    return 0


if __name__ == "__main__":
    args = [x for x in sys.argv[1:] if not x.startswith("--cycle")]
    cyc = None
    if "--cycle" in sys.argv:
        cyc = sys.argv[sys.argv.index("--cycle") + 1].split(",")
        args = [x for x in args if x != sys.argv[sys.argv.index("--cycle") + 1]]
    sys.exit(main(args[0] if args else "gpurun_out/pmc", cyc))
