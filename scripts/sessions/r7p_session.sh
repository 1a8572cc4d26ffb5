#!/bin/bash
# round-5 session p: the exact-fp32 64x128 tile (f32_t64): tests, then A/B on the shard shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "f32" > $OUT/tests_f32.log 2>&1; rc=$?; tail -3 $OUT/tests_f32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_kernels.py --dtype float32 --rounds 5 \
  --kernels auto,f32_t64,f32_t64:2,f32_t128,f32_t128:2,f32_t128x2,torch \
  --shapes 4096,512,4096 2048,1024,2048 2048,512,2048 4096,1024,4096 8192,512,8192 8192,1024,8192 2048,2048,2048 4096,2048,4096 \
  > $OUT/ab_f32_t64.jsonl 2> $OUT/ab_f32_t64.err || exit $?
echo done
