#!/bin/bash
# round-5 session am: the small-grid split rules (slot latency, T128 x 3 below
# 32 K-tiles per slice) extended to fp8 T128 — auto vs both off, settled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7am; mkdir -p $OUT
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 3 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,auto@PDMB_SPLIT_SLOT_LAT=0,auto@PDMB_SPLIT3_SMALL=0,torch \
  --shapes 768,768,8192 512,512,8192 1024,1024,16384 128,1024,8192 256,256,4096 384,768,4096 \
           384,2048,8192 512,1536,8192 640,640,16384 768,384,4096 1024,768,8192 1536,256,8192 \
           2048,512,16384 256,2048,16384 1024,256,4096 512,1024,8192 \
  > $OUT/ab_fp8_small_rules.jsonl 2> $OUT/ab.err || exit $?
echo done
