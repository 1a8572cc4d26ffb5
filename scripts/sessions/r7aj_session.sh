#!/bin/bash
# round-5 session aj: the bf16 / fp16 split slot-latency term (PDMB_SPLIT_SLOT_LAT)
# on small grids of 4-64 128^2 tiles: auto vs the switch off vs forced T128 splits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7aj; mkdir -p $OUT
for dt in bfloat16 float16; do
timeout -k 10 600 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_SPLIT_SLOT_LAT=0,t128:1,t128:2,t128:3,t128:4,torch \
  --shapes 256,256,2048 256,512,4096 384,768,4096 512,512,8192 512,1024,4096 768,768,4096 \
           1024,512,8192 256,1024,2048 1024,1024,2048 512,768,8192 1024,1024,8192 512,2048,8192 \
           768,768,8192 2048,256,8192 \
  > $OUT/ab_${dt}_slot_lat.jsonl 2> $OUT/ab_${dt}.err || exit $?
echo $dt done
done
