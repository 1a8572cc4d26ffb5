#!/bin/bash
# round-5 session al: fp8 small / thin grids, every forced tile x split arm
# against auto and hipBLASLt (settled arms), to find plans the model misses
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7al; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 3 --iters 20 --settle 1 --sessions 1 \
  --kernels auto,torch,fp8_t128:1,fp8_t128:2,fp8_t128:3,fp8_t128:4,fp8_t256x128:1,fp8_t256x128:2,fp8_t256x128:4,fp8_w4:1,fp8_w4:2,fp8_w4:4,fp8_t192:1,fp8_t192:2,fp8_t192x128:1,fp8_t192x128:2 \
  --shapes 1024,1024,4096 1024,1024,8192 512,2048,8192 768,768,8192 2048,512,4096 1536,1536,4096 \
           2048,2048,2048 1024,3072,4096 4096,512,8192 2048,1024,16384 512,512,8192 768,768,4096 \
  > $OUT/ab_fp8_small_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
