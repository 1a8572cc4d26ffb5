#!/bin/bash
# round-5 session ap: f32_t64x2 in auto — auto vs PDMB_F32T64X2=0 vs hipBLASLt
# on 20 grids drawn at random from the 121 (of 980) whose plan it changes, plus
# 4 from r7ao; settled arms, two sessions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ap; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_F32T64X2=0,torch \
  --shapes 1536,2048,2048 768,6144,4096 1536,6144,4096 3072,3072,1024 512,5120,8192 512,6144,4096 \
           6144,512,4096 2560,5120,4096 768,3072,4096 1536,3072,8192 3072,768,8192 512,5120,16384 \
           12288,256,4096 2560,2048,4096 1024,2560,2048 512,5120,2048 768,3072,2048 2048,2560,1024 \
           2048,1536,2048 512,6144,2048 1536,1536,4096 1536,3072,1024 9216,256,16384 1536,1024,4096 \
  > $OUT/ab_f32_t64x2_auto.jsonl 2> $OUT/ab.err || exit $?
echo done
