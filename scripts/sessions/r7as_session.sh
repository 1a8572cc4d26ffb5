#!/bin/bash
# round-5 session as: f32_t64x2 on the full fp32 grids (PDMB_F32T64X2_FULL=1)
# vs the current plans (f32_t128x2 / split tails) and hipBLASLt, settled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7as; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_F32T64X2_FULL=1,torch \
  --shapes 2048,4608,4096 2560,3584,8192 2560,5120,4096 2560,10240,8192 3072,3072,4096 3072,3584,4096 \
           3072,7168,8192 3584,3584,4096 3584,7168,8192 4608,4608,4096 5120,2560,8192 5120,5120,4096 \
           5120,5120,8192 7168,3072,16384 7168,3584,4096 10240,2560,4096 4608,4608,2048 \
  > $OUT/ab_f32_t64x2_full.jsonl 2> $OUT/ab.err || exit $?
echo done
