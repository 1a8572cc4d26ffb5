#!/bin/bash
# Round 6 session ZJ (PDMB_EXPERIMENTS=1 build): does the thin 256-tile round
# that follows a wide / tall grid's aspect (x_fp8_w4s_thin / x_w4s_thin: each
# XCD keeps its 8 B- (or A-) panels across the rounds) close fp8's mid-K gap on
# 4096 x 16384 x 1024 (0.90 of hipBLASLt, profiles/r8j)? Exactness screen, then
# a settled A/B against the shipping W4S and hipBLASLt, two sessions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8zj; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench > $OUT/build.log 2>&1 || exit $?
timeout -k 10 300 python scripts/check_thin.py > $OUT/check.jsonl 2> $OUT/check.err || { tail -5 $OUT/check.jsonl; tail -5 $OUT/check.err; exit 1; }
tail -1 $OUT/check.jsonl
timeout -k 10 700 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels fp8_w4s,x_fp8_w4s_thin,torch --shapes 4096,16384,1024 16384,4096,1024 4096,16384,2048 \
  2048,16384,1024 4096,16384,4096 16384,2048,1024 > $OUT/ab_fp8.jsonl 2> $OUT/ab_fp8.err || exit $?
grep '"summary"' $OUT/ab_fp8.jsonl | cut -c1-200
timeout -k 10 700 python scripts/ab_kernels.py --dtype bfloat16 --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels w4s,x_w4s_thin,torch --shapes 4096,16384,1024 4096,16384,4096 16384,4096,4096 2048,16384,4096 \
  > $OUT/ab_bf16.jsonl 2> $OUT/ab_bf16.err || exit $?
grep '"summary"' $OUT/ab_bf16.jsonl | cut -c1-200
echo "exit 0"
