#!/bin/bash
# Round 6 session Y (shipping build): f32_w4l — the lean exact-fp32 W4 K-loop
# (the experiments' x_f32_w4_lean2, not streamed) as auto's kernel on exactly
# one whole wave of 256x256 tiles (K >= 4096). Cold first launches, one per
# fresh process; the fp32 GPU tests; the exact-integer race screen; then auto
# vs the plans it replaced (f32_t128x2, f32_256s) vs hipBLASLt, settled, two
# sessions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8y; mkdir -p $OUT
for s in "4096 4096 4096" "8192 2048 8192" "4096 4096 16384" "1024 16384 16384" "2048 2048 4096 4" "4096 4096 4128" \
         "8192 2048 8192" "4096 4096 4096"; do
  timeout -k 5 45 python scripts/w4s_probe.py $s --kernel auto >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe $s rc=$?"; cat $OUT/probe.jsonl; exit 1; }
done
cut -c1-200 $OUT/probe.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "f32" > $OUT/pytest_f32.log 2>&1 || { tail -30 $OUT/pytest_f32.log; exit 1; }
tail -2 $OUT/pytest_f32.log
timeout -k 10 300 python scripts/race_screen.py --reps 50 --kernels f32_w4l > $OUT/race_f32_w4l.jsonl 2>&1 || exit $?
cut -c1-150 $OUT/race_f32_w4l.jsonl
timeout -k 10 600 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,f32_t128x2:1,f32_256s,torch --shapes 4096,4096,4096 8192,2048,8192 4096,4096,16384 \
  1024,16384,16384 2048,8192,8192 4096,4096,8192 > $OUT/ab_one_wave.jsonl 2> $OUT/ab_one_wave.err || exit $?
grep '"summary"' $OUT/ab_one_wave.jsonl | cut -c1-170
echo "exit 0"
