#!/bin/bash
# round-5 session x: exact fp32 on the VERDICT r4 #3 grids + 8k / 16k, auto vs hipBLASLt, 2 sessions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7x; mkdir -p $OUT
timeout -k 10 1100 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --sessions 2 --kernels auto,torch \
  --shapes 1024,16384,16384 16384,1024,16384 4096,4096,14336 2048,8192,8192 8192,2048,8192 4096,12288,12288 \
           8192,8192,28672 8192,8192,8192 16384,16384,16384 \
  > $OUT/ab_f32_verdict3.jsonl 2> $OUT/ab_f32_verdict3.err || exit $?
grep summary $OUT/ab_f32_verdict3.jsonl | cut -c1-220
bash scripts/gpu_session.sh r7x final_table
