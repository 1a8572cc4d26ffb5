#!/bin/bash
# Wave-quantisation tail: GEMM/mode/overlap tests, then auto vs hipBLASLt on shapes
# whose last 256x256 wave is mostly empty, and a full-chip control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2tail}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_modes_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels w4:1,auto,torch \
  --shapes 6000,6000,6144 6144,6144,6144 3000,7000,5056 10000,10000,10048 5000,5000,5056 7168,7168,7168 12288,12288,12288 > $OUT/ab.log 2>&1
rc=$?; cut -c1-110 $OUT/ab.log | tail -21; exit $rc
