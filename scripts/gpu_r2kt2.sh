#!/bin/bash
# After the T256x128 kt refit: GEMM/mode tests, then auto vs the explicit kernels and hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2kt2}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_modes_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels w4,t256x128,auto,torch \
  --shapes 3000,7000,5056 8192,1024,8192 4096,2048,4096 2000,3000,4096 6000,6000,6144 > $OUT/ab.log 2>&1
rc=$?; cut -c1-110 $OUT/ab.log | tail -20; exit $rc
