#!/bin/bash
# round-5 session ad: exact-fp32 small / thin grids that still trail hipBLASLt —
# every forced split arm of f32_t128 / f32_t64 / f32_t128x2 against auto, to
# refit the split-K terms of the cost model (arms a K cannot take are skipped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ad; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --sessions 1 \
  --kernels auto,torch,f32_t128:1,f32_t128:2,f32_t128:3,f32_t128:4,f32_t128:5,f32_t128:6,f32_t128:8,f32_t64:1,f32_t64:2,f32_t64:3,f32_t64:4,f32_t64:6,f32_t64:8,f32_t128x2:1,f32_t128x2:2,f32_t128x2:3,f32_t128x2:4,f32_t128x2:6,f32_t128x2:8 \
  --shapes 1536,3072,1024 2560,512,8192 1024,1024,4096 2048,512,2048 \
           3072,256,16384 1024,256,16384 9216,256,16384 2048,256,8192 4096,1024,4096 2048,2048,2048 \
  > $OUT/ab_f32_small_split_arms2.jsonl 2> $OUT/ab2.err || exit $?
echo done
