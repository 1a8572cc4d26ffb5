#!/bin/bash
# Round-2 pass W (experiment build): tile family with the epilogue folded into the last K-tile vs
# the unfused kernels (x_t128_unfused, x_fp8_t128_unfused) and hipBLASLt; tile/fp8 exactness tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2w}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_overlap_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --rounds 7 --kernels t128:1,x_t128_unfused,t256x128:1,auto,torch \
  --shapes 2048,2048,2048 4096,1024,4096 4096,512,4096 4096,2048,4096 > $OUT/ab_bf16.log 2>&1
rc=$?; tail -20 $OUT/ab_bf16.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 7 --kernels fp8_t128:1,x_fp8_t128_unfused,auto,torch \
  --shapes 2048,2048,2048 4096,1024,4096 4096,512,4096 > $OUT/ab_fp8.log 2>&1
rc=$?; tail -12 $OUT/ab_fp8.log | cut -c1-150; exit $rc
