#!/bin/bash
# Round-2 pass S: exact-fp32 W4 split-K for under-filled grids (tests + auto vs hipBLASLt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2s}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py tests/test_modes_gpu.py -x -q --timeout 120 --timeout-method thread -k "f32 or fp32" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --dtype float32 --rounds 5 --iters 8 \
  --kernels auto,f32_w4,f32_256s,torch --shapes 4096,2048,4096 4096,1024,4096 4096,512,4096 2048,2048,2048 8192,1024,8192 4096,4096,4096 8192,8192,8192 > $OUT/ab.log 2>&1
rc=$?; tail -28 $OUT/ab.log | cut -c1-150; exit $rc
