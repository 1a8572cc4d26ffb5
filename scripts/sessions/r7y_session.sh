#!/bin/bash
# round-5 session y: race screen of the non-power-of-two split plans and the 64x128 fp32 tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7y; mkdir -p $OUT
timeout -k 10 900 python scripts/race_screen.py --splits --reps 50 > $OUT/race_splits.jsonl 2> $OUT/race_splits.err || exit $?
timeout -k 10 600 python scripts/race_screen.py --kernels f32_t64 --reps 100 > $OUT/race_f32_t64.jsonl 2> $OUT/race_f32_t64.err || exit $?
cat $OUT/race_splits.jsonl $OUT/race_f32_t64.jsonl | cut -c1-260
