#!/usr/bin/env python3
"""Per-kernel instruction statistics of a hipcc ``-save-temps`` gfx950 ``.s`` file:
MFMA / ds_read / LDS-DMA / barrier counts, the s_waitcnt histogram (look for
vmcnt(0) inside the K-loop) and the register budget.

    hipcc --offload-arch=gfx950 -O3 -save-temps -c k.hip && python scripts/asm_stats.py *gfx950*.s
"""
import re
import sys
from collections import Counter


def main(paths):
    for p in paths:
        s = open(p).read()
        for m in re.finditer(r"^([A-Za-z_][\w.$]*):\s*;\s*@", s, re.M):
            name = m.group(1)
            end = s.find(".Lfunc_end", m.end())
            body = s[m.end():end]
            nv = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s)
            print(f"{name}: lines={body.count(chr(10))} vgpr={nv.group(1) if nv else '?'} "
                  f"mfma={len(re.findall('v_mfma', body))} ds_read={len(re.findall('ds_read', body))} "
                  f"dma={len(re.findall(r'buffer_load_dwordx4.*lds', body))} "
                  f"barrier={body.count('s_barrier')} spill={'scratch_' in body}")
            print("   waits:", Counter(re.findall(r"s_waitcnt [^\n;]*", body)).most_common(14))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
