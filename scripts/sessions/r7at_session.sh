#!/bin/bash
# round-5 session at: f32_t64x2 split on the full fp32 grids without a split
# tail (the rule as built after r7as) — auto vs PDMB_F32T64X2_FULL=0, settled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7at; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_F32T64X2_FULL=0,torch \
  --shapes 2560,5120,2048 2560,5120,16384 3072,3584,4096 3072,3584,16384 3072,7168,4096 3584,3072,4096 \
           3584,3584,2048 3584,3584,8192 3584,6144,8192 4608,4608,8192 4608,4608,16384 5120,2560,2048 \
           5120,2560,4096 6144,3584,4096 7168,3072,8192 6144,3584,16384 \
  > $OUT/ab_f32_t64x2_full_rule.jsonl 2> $OUT/ab.err || exit $?
echo done
