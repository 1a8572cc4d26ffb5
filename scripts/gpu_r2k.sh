#!/bin/bash
# Round-2 pass K: batched (bmm of 4) vs single 16k W4S, and fp8 T128 split-K arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2k}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels auto,w4,torch \
  --shapes 16384,16384,16384 16384,16384,16384,4 16384,16384,16384,2 > $OUT/bmm_ab.log 2>&1
rc=$?; tail -12 $OUT/bmm_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 \
  --kernels fp8_t128:1,fp8_t128:2,fp8_t128:4,auto,torch \
  --shapes 4096,512,4096 2048,2048,2048 4096,1024,4096 2048,1024,8192 > $OUT/fp8_split.log 2>&1
rc=$?; tail -24 $OUT/fp8_split.log; exit $rc
