#!/bin/bash
# round-5 session ak: T128 x 3 on bf16 / fp16 grids of <= 36 tiles with
# 8-31 K-tiles per slice (PDMB_SPLIT3_SMALL) — auto vs the rule off, settled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ak; mkdir -p $OUT
for dt in bfloat16 float16; do
timeout -k 10 600 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_SPLIT3_SMALL=0,t128:1,t128:2,t128:3,torch \
  --shapes 128,128,4096 128,1024,2048 256,256,4096 256,768,2048 384,384,4096 384,640,2048 \
           512,512,4096 512,512,2048 640,768,4096 768,768,4096 768,256,2048 1024,512,4096 \
           1024,128,2048 512,1024,4096 256,1024,4096 640,384,2048 \
  > $OUT/ab_${dt}_split3_small.jsonl 2> $OUT/ab_${dt}.err || exit $?
echo $dt done
done
