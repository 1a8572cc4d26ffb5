#!/bin/bash
# Round 6 session D (PDMB_EXPERIMENTS=1 build in the tree): fp8 short-K grids
# (VERDICT r5 #4), which are write-bound. Plain (temporal) vs the shipping
# non-temporal C stores, and the W4S stream down to four K-tiles (x_fp8_w4s_k4),
# which overlaps a tile's C stores with the next tile's K-loop. Arms against
# hipBLASLt in the same processes, settled, two sessions. First: the write
# bandwidth a plain fill / copy of the 512 MiB output reaches on this box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8d; mkdir -p $OUT
echo "== build $(date +%T)"
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== write bandwidth $(date +%T)"
timeout -k 10 120 python - > $OUT/write_bw.jsonl 2> $OUT/write_bw.err <<'PY' || exit $?
import json, torch
C = torch.empty(16384, 16384, device="cuda", dtype=torch.bfloat16)
D = torch.randn(16384, 16384, device="cuda", dtype=torch.bfloat16)
for name, fn, moved in (("fill", lambda: C.fill_(1.0), C.nbytes), ("copy", lambda: C.copy_(D), 2 * C.nbytes)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print(json.dumps({"op": name, "bytes_moved": moved, "us": round(us, 1), "TB_per_s": round(moved / us / 1e6, 3)}))
PY
cat $OUT/write_bw.jsonl
echo "== fp8 short K $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels fp8_w4,x_fp8_w4_tstore,x_fp8_w4s_k4,x_fp8_w4s_k4_tstore,auto,torch \
  --shapes 16384,16384,512 8192,8192,512 16384,8192,512 4096,4096,512 \
  > $OUT/ab_fp8_k512.jsonl 2> $OUT/ab_fp8_k512.err || exit $?
grep -v '"session"' $OUT/ab_fp8_k512.jsonl | cut -c1-220
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels fp8_w4,fp8_w4s,x_fp8_w4s_tstore,x_fp8_w4s_k4,auto,torch \
  --shapes 16384,16384,1024 8192,8192,1024 \
  > $OUT/ab_fp8_k1024.jsonl 2> $OUT/ab_fp8_k1024.err || exit $?
grep -v '"session"' $OUT/ab_fp8_k1024.jsonl | cut -c1-220
echo "exit 0"
