#!/bin/bash
# Round 6 session ZA (shipping build): f32_w4l (the lean exact-fp32 W4 loop)
# forced on multi-wave fp32 grids of whole 256x256 tiles, against the plan auto
# runs there (f32_t128x2 unsplit) and hipBLASLt; settled, two sessions. Does
# the one-wave rule extend to every whole-wave grid with K >= 4096?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8za; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 3 --settle 1 --sessions 2 \
  --kernels f32_t128x2:1,f32_w4l,torch --shapes 8192,8192,8192 16384,16384,16384 16384,8192,16384 \
  16384,4096,16384 16384,2048,16384 8192,4096,8192 12288,12288,12288 8192,8192,4096 4096,4096,4096,2 \
  > $OUT/ab_multi_wave.jsonl 2> $OUT/ab_multi_wave.err || exit $?
grep '"summary"' $OUT/ab_multi_wave.jsonl | cut -c1-170
echo "exit 0"
