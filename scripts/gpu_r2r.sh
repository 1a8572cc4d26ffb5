#!/bin/bash
# Round-2 pass R (experiment build): fp32 f32_256s with the LDS-staged non-temporal epilogue vs its
# direct-store form (x_f32_256s_direct), f32_w4 and hipBLASLt; fp32 exactness tests incl. edges.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2r}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py tests/test_modes_gpu.py -x -q --timeout 120 --timeout-method thread -k "f32 or fp32" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab_kernels.py --dtype float32 --rounds 7 --iters 8 \
  --kernels f32_256s,x_f32_256s_direct,f32_w4,torch --shapes 4096,4096,4096 8192,8192,8192 16384,16384,16384 4096,2048,4096 > $OUT/ab.log 2>&1
rc=$?; tail -16 $OUT/ab.log | cut -c1-160; exit $rc
