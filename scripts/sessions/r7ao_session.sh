#!/bin/bash
# round-5 session ao: exact-fp32 f32_t64x2 (64x128 tile, 2 stages, two per CU):
# exactness tests, then forced split arms and auto with it priced
# (PDMB_F32T64X2=1) on the fp32 grids that still trail hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ao; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "f32" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 1 \
  --kernels auto,auto@PDMB_F32T64X2=1,torch,f32_t64:2,f32_t64:3,f32_t64:4,f32_t64x2:1,f32_t64x2:2,f32_t64x2:3,f32_t64x2:4,f32_t64x2:6,f32_t64x2:8,f32_t128:3,f32_t128:5 \
  --shapes 1536,1536,4096 2560,512,8192 1024,1024,4096 2048,512,2048 9216,256,16384 2048,256,8192 \
           1536,3072,1024 1024,2048,4096 3072,512,4096 4096,512,4096 1536,1024,4096 512,3072,4096 \
  > $OUT/ab_f32_t64x2_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
