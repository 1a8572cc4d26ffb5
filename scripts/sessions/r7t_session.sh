#!/bin/bash
# round-5 session t: the 3-way split on the wider set of grids auto now gives it (bf16, fp32), 2 sessions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7t; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype bfloat16 --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 4608,2048,16384 9216,1024,16384 3584,2560,16384 1024,9216,16384 2560,3584,16384 512,9216,16384 \
           1024,2560,16384 3584,512,16384 1536,6656,16384 \
  > $OUT/ab_bf16.jsonl 2> $OUT/ab_bf16.err || exit $?
timeout -k 10 300 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 --kernels auto,auto@PDMB_SPLIT3=0,torch \
  --shapes 2304,2304,4096 1536,1536,8192 5120,256,8192 > $OUT/ab_f32.jsonl 2> $OUT/ab_f32.err || exit $?
echo done
