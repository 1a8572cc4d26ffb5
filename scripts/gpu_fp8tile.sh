#!/bin/bash
# fp8 tile family: GPU tests, then an interleaved A/B vs fp8 W4 (planner split) and hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fp8tile}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 \
  --kernels fp8_w4,fp8_t128,fp8_t128:1,fp8_t256x128,auto,torch \
  --shapes 4096,512,4096 4096,1024,4096 2048,2048,2048 4096,2048,4096 8192,1024,8192 4096,4096,4096 8192,2048,8192 \
  > $OUT/ab.log 2>&1
rc=$?; tail -60 $OUT/ab.log; exit $rc
