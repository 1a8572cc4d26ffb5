#!/bin/bash
# Round 6 session ZG (shipping build): fp8 e4m3 matrix_parallel shards at
# ws = 2 / 4 / 8 of the reference's default sizes (the MI355X dtype extension),
# auto vs hipBLASLt (_scaled_mm), settled, two sessions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8zg; mkdir -p $OUT
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels auto,torch --shapes 4096,2048,4096 4096,1024,4096 4096,512,4096 8192,4096,8192 8192,2048,8192 \
  8192,1024,8192 16384,8192,16384 16384,4096,16384 16384,2048,16384 \
  > $OUT/shards_fp8.jsonl 2> $OUT/shards_fp8.err || exit $?
grep '"summary"' $OUT/shards_fp8.jsonl | cut -c1-170
echo "exit 0"
