#!/bin/bash
# round-5 session af: confirmation of the fp32 planner change (8-way split on
# f32_t64 only, split f32_t128x2 on grids of < 2 tiles per CU) on 21 new grids
# plus the 6 grids r7ae found mixed; rounds = 4 = arms, so every arm takes
# every position once, and each timed run follows an untimed run of the same
# arm (--settle 1: the arm right after hipBLASLt measured up to 3 % low)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7af; mkdir -p $OUT
timeout -k 10 1000 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_F32X2SPLIT=0,auto@PDMB_SPLIT8=0,torch \
  --shapes 4096,768,16384 1024,5120,4096 6144,768,8192 3072,2048,1024 12288,512,4096 8192,768,16384 \
           6144,512,2048 256,12288,2048 4096,1024,16384 768,256,16384 256,768,8192 1536,5120,8192 \
           2560,3072,4096 768,6144,2048 3072,1536,2048 1536,512,16384 256,3072,16384 6144,768,16384 \
           768,6144,16384 2560,2560,16384 2560,2560,4096 \
           512,9216,16384 512,3072,8192 512,1024,16384 1024,4096,16384 2560,3072,8192 3072,256,16384 \
  > $OUT/ab_f32_planner_confirm_settled.jsonl 2> $OUT/ab.err || exit $?
echo done
