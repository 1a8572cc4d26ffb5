#!/bin/bash
# Round 6 session ZE (shipping build, final kernels: f32_w4l, lean f32_t128, padded W4S): the closing dtype table again, auto vs hipBLASLt
# at the reference's default sizes (4096 / 8192 / 16384), every dtype, settled,
# position-balanced arms, two sessions; then matrix_parallel's shard shapes at
# ws = 2 / 4 / 8 for bf16 and exact fp32 (the reference's dtype surface).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8ze; mkdir -p $OUT
for dt in bfloat16 float16 float8_e4m3fn float32; do
  it=20; [ $dt = float32 ] && it=5
  timeout -k 10 400 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters $it --settle 1 --sessions 2 \
    --kernels auto,torch --sizes 4096 8192 16384 > $OUT/table_$dt.jsonl 2> $OUT/table_$dt.err || exit $?
  grep '"summary"' $OUT/table_$dt.jsonl | cut -c1-160
done
for dt in bfloat16 float32; do
  it=20; [ $dt = float32 ] && it=5
  timeout -k 10 500 python scripts/ab_kernels.py --dtype $dt --rounds 4 --iters $it --settle 1 --sessions 2 \
    --kernels auto,torch --shapes 4096,2048,4096 4096,1024,4096 4096,512,4096 8192,4096,8192 8192,2048,8192 \
    8192,1024,8192 16384,8192,16384 16384,4096,16384 16384,2048,16384 \
    > $OUT/shards_$dt.jsonl 2> $OUT/shards_$dt.err || exit $?
  grep '"summary"' $OUT/shards_$dt.jsonl | cut -c1-160
done
echo "exit 0"
