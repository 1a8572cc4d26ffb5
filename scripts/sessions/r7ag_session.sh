#!/bin/bash
# round-5 session ag: GPU tests of the fp32 planner change (exact-integer /
# edge / bitwise), then the race screen over auto's split plans incl. the new ones
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ag; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "f32 or splitk or split3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python scripts/race_screen.py --splits --reps 50 > $OUT/race_splits.jsonl 2> $OUT/race.err || exit $?
echo done
