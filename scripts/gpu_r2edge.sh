#!/bin/bash
# W4 edge tiles (masked epilogue) and the K-only padded path writing C in place: GEMM tests, then
# auto vs hipBLASLt on shapes off the 256 grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2edge}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_modes_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels auto,torch --shapes 5000,5000,5000 \
  10000,10000,10000 12345,12345,12345 3000,7000,5000 8192,8192,1000 16000,16000,16000 6000,6000,6144 > $OUT/ab.log 2>&1
rc=$?; tail -14 $OUT/ab.log | cut -c1-130; exit $rc
