#!/bin/bash
# round-5 session au: GPU tests (gemm / fp8 / modes) and the split race screen
# after the full-grid f32_t64x2 rule
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7au; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_modes_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python scripts/race_screen.py --splits --reps 30 > $OUT/race_splits.jsonl 2> $OUT/race.err || exit $?
echo done
