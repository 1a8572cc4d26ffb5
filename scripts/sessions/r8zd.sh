#!/bin/bash
# Round 6 session ZD (shipping build): unsplit f32_t128 on the lean K-loop.
# Cold first launches; exact-integer race screen; auto vs hipBLASLt on the
# grids auto runs it on (settled, two sessions); then closing validation D:
# the whole GPU suite, smoke, bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8zd; mkdir -p $OUT
for s in "4096 1024 4096" "2048 2048 2048" "1000 1052 4096"; do
  timeout -k 5 45 python scripts/w4s_probe.py $s --kernel auto >> $OUT/probe.jsonl 2>> $OUT/probe.err || { echo "probe $s rc=$?"; cat $OUT/probe.jsonl; exit 1; }
done
cut -c1-200 $OUT/probe.jsonl
timeout -k 10 300 python scripts/race_screen.py --reps 50 --kernels f32_t128 > $OUT/race_f32_t128.jsonl 2>&1 || exit $?
cut -c1-150 $OUT/race_f32_t128.jsonl
timeout -k 10 500 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels auto,torch --shapes 4096,1024,4096 2048,2048,2048 4096,2048,4096 4096,512,4096 \
  > $OUT/ab_t128.jsonl 2> $OUT/ab_t128.err || exit $?
grep '"summary"' $OUT/ab_t128.jsonl | cut -c1-170
bash scripts/gpu_session.sh r8zd tests smoke bench rocprof_bench || exit $?
echo "exit 0"
