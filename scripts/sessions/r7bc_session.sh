#!/bin/bash
# round-5 session bc: fp8 W4 vs W4S at 2-3 tiles per CU and short K (the W4S
# rule takes it from 2 per CU at any K)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7bc; mkdir -p $OUT
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,fp8_w4,fp8_w4s,torch \
  --shapes 8192,4096,1024 4096,8192,1024 16384,2048,1024 8192,4096,2048 4096,8192,2048 8192,4096,4096 \
           12288,4096,1024 8192,6144,1024 12288,4096,2048 8192,8192,1024 \
  > $OUT/ab_fp8_w4_vs_w4s_short_k.jsonl 2> $OUT/ab.err || exit $?
echo done
