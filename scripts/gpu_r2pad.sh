#!/bin/bash
# Vectorised pad_copy: GEMM / mode tests (padded path included), then padded shapes vs hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2pad}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_modes_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels auto,torch \
  --shapes 6000,6000,6100 12345,12345,12345 8192,8192,1000 4000,4000,4000 > $OUT/ab.log 2>&1
rc=$?; cut -c1-110 $OUT/ab.log | tail -8; exit $rc
