#!/bin/bash
# round-5 session u: 5- / 6-way split-K (PDMB_SPLIT56=1) vs the current auto vs hipBLASLt, 2 sessions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "splitk or tiled_random" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_kernels.py --dtype bfloat16 --rounds 5 --sessions 2 --kernels auto@PDMB_SPLIT56=1,auto,torch \
  --shapes 512,256,16384 1024,256,16384 2560,256,16384 512,5632,16384 4608,256,16384 3072,256,16384 \
  > $OUT/ab_bf16.jsonl 2> $OUT/ab_bf16.err || exit $?
timeout -k 10 600 python scripts/ab_kernels.py --dtype float32 --rounds 5 --sessions 2 --kernels auto@PDMB_SPLIT56=1,auto,torch \
  --shapes 512,6400,16384 1024,3328,16384 3072,256,16384 9216,256,16384 1024,256,16384 3072,4864,16384 \
  > $OUT/ab_f32.jsonl 2> $OUT/ab_f32.err || exit $?
echo done
