#!/bin/bash
# round-5 session ar: exact-fp32 mid grids (1-3 waves of 128^2 tiles at two
# per CU), every kernel x split arm against auto and hipBLASLt (settled)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ar; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 1 \
  --kernels auto,torch,f32_t128x2:1,f32_t128x2:2,f32_t128:1,f32_t128:2,f32_t64x2:1,f32_t64x2:2,f32_t64x2:4,f32_256s,f32_w4:1,f32_w4:2 \
  --shapes 3072,3072,4096 2560,4096,4096 4608,4608,2048 3584,3584,4096 5120,2048,4096 6144,2048,4096 \
           2048,6144,8192 4096,3072,4096 3072,4096,8192 2560,2560,8192 \
  > $OUT/ab_f32_mid_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
