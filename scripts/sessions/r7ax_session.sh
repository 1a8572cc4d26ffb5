#!/bin/bash
# round-5 session ax: fp16 at the default sizes and the small-grid planner grids,
# settled arms (the bf16 / fp32 / fp8 counterparts are r7ah)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ax; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float16 --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels auto,torch \
  --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 3072,3072,3072 8192,2048,8192 16384,2048,16384 \
           4096,512,4096 1024,1024,8192 768,768,4096 \
  > $OUT/ab_fp16_table_settled.jsonl 2> $OUT/ab.err || exit $?
echo done
