#!/bin/bash
# round-5 session e: 192-row tiles — correctness, then A/B against the incumbents and hipBLASLt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; export TMPDIR=/tmp; OUT=gpurun_out/r7e; mkdir -p $OUT
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
echo "== tests $(date +%T)"
timeout -k 10 600 $PYT tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu -k "t192 or tile_family" > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== ab bf16 $(date +%T)"
timeout -k 10 600 python scripts/ab_kernels.py --dtype bfloat16 --rounds 5 --kernels auto,t192,t192x128,w4,t256x128,torch \
  --shapes 3072,3072,3072 2304,2304,4096 6144,6144,6144 4608,4608,3072 3072,8192,3072 1536,1536,4096 > $OUT/ab_bf16.log 2>&1 || exit $?
grep '^{' $OUT/ab_bf16.log > $OUT/ab_bf16.jsonl
echo "== ab fp8 $(date +%T)"
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 --kernels auto,fp8_t192,fp8_t192x128,fp8_w4,fp8_t256x128,torch \
  --shapes 3072,3072,3072 2304,2304,4096 4608,4608,3072 3072,8192,3072 5120,5120,4096 > $OUT/ab_fp8.log 2>&1 || exit $?
grep '^{' $OUT/ab_fp8.log > $OUT/ab_fp8.jsonl
echo "== done $(date +%T)"
