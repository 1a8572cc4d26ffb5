#!/bin/bash
# round-5 session q: f32_t64 on the grids auto now gives it (auto vs PDMB_F32T64=0 vs hipBLASLt), 2 sessions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7q; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 \
  --kernels auto,auto@PDMB_F32T64=0,torch \
  --shapes 4096,512,4096 2048,1024,2048 2048,512,2048 4096,256,4096 8192,256,4096 1024,2048,4096 1536,1024,4096 \
           3072,512,4096 512,3072,4096 1024,1024,4096 2048,256,8192 6144,256,8192 2560,512,8192 4096,512,1024 \
  > $OUT/ab_f32_t64_auto.jsonl 2> $OUT/ab_f32_t64_auto.err || exit $?
echo done
