#!/bin/bash
# Round-2 pass T (experiment build): fp8 W4 with the epilogue folded into the last K-tile vs the
# unfused kernel (x_fp8_w4_unfused) and hipBLASLt; fp8 exactness tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2t}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 7 \
  --kernels fp8_w4,x_fp8_w4_unfused,torch --shapes 4096,4096,4096 8192,2048,8192 4096,8192,4096 2048,8192,8192 > $OUT/ab.log 2>&1
rc=$?; tail -12 $OUT/ab.log | cut -c1-150; exit $rc
