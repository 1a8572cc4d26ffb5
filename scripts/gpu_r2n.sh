#!/bin/bash
# Round-2 pass N (experiment build, PDMB_EXPERIMENTS=1): non-temporal C stores (hipBLASLt's fp8
# kernels are NTD) vs the shipping epilogue: fp8 W4 at one 256^2 tile per CU, fp8 W4S, bf16 W4S.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2n}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 7 \
  --kernels fp8_w4,x_fp8_w4_ntstore,torch \
  --shapes 4096,4096,4096 8192,2048,8192 4096,8192,4096 > $OUT/fp8_w4.log 2>&1
rc=$?; tail -9 $OUT/fp8_w4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 7 \
  --kernels fp8_w4s,x_fp8_w4s_ntstore,torch --shapes 8192,8192,8192 16384,16384,16384 16384,16384,2048 > $OUT/fp8_w4s.log 2>&1
rc=$?; tail -9 $OUT/fp8_w4s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --rounds 7 --iters 10 \
  --kernels w4s,x_w4s_ntstore --shapes 16384,16384,16384 8192,8192,8192 16384,16384,2048 > $OUT/w4s.log 2>&1
rc=$?; tail -6 $OUT/w4s.log; exit $rc
