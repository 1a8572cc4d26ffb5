#!/bin/bash
# round-5 session av: bf16 mid grids (1-3 waves of 256^2 tiles), every kernel x
# split arm against auto and hipBLASLt (settled)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7av; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype bfloat16 --rounds 3 --iters 10 --settle 1 --sessions 1 \
  --kernels auto,torch,w4:1,w4:2,w4s,t256x128:1,t256x128:2,t128:1,t128:2,t128x2:1,t128x2:2,t192:1,t192:2,t192x128:1,t192x128:2 \
  --shapes 2560,4096,4096 3584,3584,4096 4608,4608,2048 5120,2048,4096 3072,4096,8192 2560,2560,8192 \
           6144,2560,4096 7168,3072,4096 3584,3584,8192 4608,4608,4096 \
  > $OUT/ab_bf16_mid_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
