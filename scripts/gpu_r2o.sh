#!/bin/bash
# Round-2 pass O: non-temporal C stores in every shipping epilogue + fp8 tile family: full validation,
# then auto vs hipBLASLt on the reference's sizes and the shard shapes (bf16, fp8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_validate.sh r2o || exit $?
OUT=gpurun_out/r2o
timeout -k 10 400 python -u scripts/ab_kernels.py --rounds 5 --kernels auto,torch \
  --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 16384,2048,16384 8192,2048,8192 8192,1024,8192 \
           4096,2048,4096 4096,1024,4096 4096,512,4096 2048,2048,2048 > $OUT/ab_bf16.log 2>&1
rc=$?; tail -20 $OUT/ab_bf16.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 --kernels auto,torch \
  --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 16384,2048,16384 8192,2048,8192 8192,1024,8192 \
           4096,2048,4096 4096,1024,4096 4096,512,4096 2048,2048,2048 > $OUT/ab_fp8.log 2>&1
rc=$?; tail -20 $OUT/ab_fp8.log | cut -c1-200; exit $rc
