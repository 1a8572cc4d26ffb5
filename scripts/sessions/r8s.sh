#!/bin/bash
# Round 6 session S (shipping build): f32_w4s promoted to a shipping kernel and
# taken by auto on whole waves of 256x256 tiles. Its GPU tests (exact, bitwise
# vs f32_w4, refusals, graph replay), the exact-integer race screen, then the
# fp32 closing table again (auto vs hipBLASLt, settled, two sessions) at the
# reference's default squares and matrix_parallel's shards.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8s; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "f32" > $OUT/pytest_f32.log 2>&1 || { tail -30 $OUT/pytest_f32.log; exit 1; }
tail -2 $OUT/pytest_f32.log
timeout -k 10 300 python scripts/race_screen.py --reps 50 --kernels f32_w4s > $OUT/race_f32_w4s.jsonl 2>&1 || exit $?
cat $OUT/race_f32_w4s.jsonl | cut -c1-160
timeout -k 10 400 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,f32_t128x2,torch --sizes 4096 8192 16384 > $OUT/table_float32.jsonl 2> $OUT/table_float32.err || exit $?
grep '"summary"' $OUT/table_float32.jsonl | cut -c1-160
timeout -k 10 500 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,torch --shapes 8192,4096,8192 8192,2048,8192 16384,8192,16384 16384,4096,16384 16384,2048,16384 \
  > $OUT/shards_float32.jsonl 2> $OUT/shards_float32.err || exit $?
grep '"summary"' $OUT/shards_float32.jsonl | cut -c1-160
echo "exit 0"
