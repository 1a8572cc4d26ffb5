#!/bin/bash
# Round 6 session G (PDMB_EXPERIMENTS=1 build in the tree): the ws = 8 shard
# grids (16384 x 2048 x 16384, 8192 x 2048 x 8192: 8 tile columns) run map_tile
# mode 3 (a 4 x 2 XCD grid of 8 x 4 blocks: 8 A + 4 B panels per XCD per
# K-step). Session r8c found 4 x 8 blocks (4 A + 8 B) 1.35 % ahead of 8 x 4 at
# 16k; supertile 9 gives the thin grids 4 x 8 blocks (an 8 x 1 XCD grid).
# bf16 and fp8, W4S and W4 arms, settled, two sessions, bitwise vs shipping.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8g; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== bf16 $(date +%T)"
timeout -k 10 500 python scripts/ab_kernels.py --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels w4s,x_w4s_st9,torch --shapes 16384,2048,16384 16384,2048,8192 32768,2048,8192 \
  > $OUT/ab_bf16_w4s.jsonl 2> $OUT/ab_bf16_w4s.err || exit $?
grep '"summary"' $OUT/ab_bf16_w4s.jsonl | cut -c1-200
timeout -k 10 400 python scripts/ab_kernels.py --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels w4,x_w4_st9,torch --shapes 8192,2048,8192 8192,2048,16384 \
  > $OUT/ab_bf16_w4.jsonl 2> $OUT/ab_bf16_w4.err || exit $?
grep '"summary"' $OUT/ab_bf16_w4.jsonl | cut -c1-200
echo "== fp8 $(date +%T)"
timeout -k 10 500 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels fp8_w4s,x_fp8_w4s_st9,torch --shapes 16384,2048,16384 16384,2048,8192 32768,2048,8192 \
  > $OUT/ab_fp8_w4s.jsonl 2> $OUT/ab_fp8_w4s.err || exit $?
grep '"summary"' $OUT/ab_fp8_w4s.jsonl | cut -c1-200
timeout -k 10 400 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels fp8_w4,x_fp8_w4_st9,torch --shapes 8192,2048,8192 8192,2048,16384 \
  > $OUT/ab_fp8_w4.jsonl 2> $OUT/ab_fp8_w4.err || exit $?
grep '"summary"' $OUT/ab_fp8_w4.jsonl | cut -c1-200
grep -h '"bitwise_eq_first": false' $OUT/ab_*.jsonl | grep -v torch | cut -c1-200
echo "== counters $(date +%T)"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
grep -o "SQ_INSTS_[A-Z0-9_]*" $OUT/counters.txt | sort -u | head -60
echo "exit 0"
