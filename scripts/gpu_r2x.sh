#!/bin/bash
# Round-2 pass X (experiment build): bf16 W4 with the epilogue folded into the last K-tile vs the
# unfused kernel (x_w4_unfused) and hipBLASLt; GEMM exactness tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2x}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_overlap_gpu.py tests/test_modes_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --rounds 7 --kernels w4:1,x_w4_unfused,auto,torch \
  --shapes 4096,4096,4096 8192,2048,8192 4096,8192,4096 8192,8192,2048 > $OUT/ab.log 2>&1
rc=$?; tail -16 $OUT/ab.log | cut -c1-150; exit $rc
