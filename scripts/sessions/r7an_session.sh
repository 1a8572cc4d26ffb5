#!/bin/bash
# round-5 session an: GPU tests of the small-grid split rules (bf16 / fp16 /
# fp8) and the fp32 planner change, then the race screen over the split plans
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7an; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "small_grid or split or f32_auto or tile_family or planner" > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python scripts/race_screen.py --splits --reps 50 > $OUT/race_splits.jsonl 2> $OUT/race.err || exit $?
echo done
