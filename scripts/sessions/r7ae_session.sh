#!/bin/bash
# round-5 session ae: the fp32 planner's 8-way split and split f32_t128x2 on
# grids of < 2 tiles per CU, A/B'd against their switches (PDMB_SPLIT8=0,
# PDMB_F32X2SPLIT=0) and hipBLASLt on a sample of the grids whose plan changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ae; mkdir -p $OUT
timeout -k 10 1000 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --sessions 2 \
  --kernels auto,auto@PDMB_F32X2SPLIT=0,auto@PDMB_SPLIT8=0,torch \
  --shapes 512,6144,4096 1024,3072,8192 2560,2048,4096 512,12288,4096 2048,3072,2048 1024,6144,16384 \
           512,6144,2048 1024,4096,16384 512,9216,16384 256,512,16384 1024,256,8192 512,3072,8192 \
           1536,5120,4096 2560,3072,8192 1536,3072,2048 768,1024,16384 512,1024,16384 2560,2560,8192 \
           3072,256,16384 1024,256,16384 \
  > $OUT/ab_f32_split8_x2split.jsonl 2> $OUT/ab.err || exit $?
echo done
