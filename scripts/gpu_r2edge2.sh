#!/bin/bash
# Tile-family edge tiles: GEMM / fp8 / mode tests, then W4 vs T256x128 vs T128 vs auto vs hipBLASLt
# on shapes whose 256^2 grids quantise badly.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2edge2}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_modes_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels w4:1,t256x128:1,t128:1,auto,torch \
  --shapes 5000,5000,5056 3000,7000,5056 6000,6000,6144 10000,10000,10048 2000,3000,4096 > $OUT/ab.log 2>&1
rc=$?; tail -25 $OUT/ab.log | cut -c1-120; exit $rc
