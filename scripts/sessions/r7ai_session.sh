#!/bin/bash
# round-5 session ai: bf16 small / thin grids, every forced tile x split arm
# against auto and hipBLASLt (settled arms), to find plans the model misses
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ai; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype bfloat16 --rounds 3 --iters 10 --settle 1 --sessions 1 \
  --kernels auto,torch,t128:1,t128:2,t128:3,t128:4,t128:8,t128x2:1,t128x2:2,t128x2:3,t128x2:4,t128x2:8,t256x128:1,t256x128:2,t256x128:4,w4:1,w4:2,w4:4,w4:8,t192:1,t192:2,t192x128:1,t192x128:2,t192x128:4 \
  --shapes 1024,1024,4096 1024,1024,8192 2048,512,4096 512,2048,8192 1536,1536,4096 2048,2048,1024 \
           1024,3072,2048 768,768,8192 2560,512,8192 4096,512,4096 1024,256,16384 3072,1024,4096 \
  > $OUT/ab_bf16_small_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
