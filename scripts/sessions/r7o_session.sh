#!/bin/bash
# round-5 session o: every fp8 arm on the sweep grids where auto trails hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7o; mkdir -p $OUT
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 \
  --kernels auto,fp8_w4,fp8_w4s,fp8_t256x128,fp8_t128,fp8_w4:2,fp8_t256x128:2,torch \
  --shapes 8192,8192,1024 4096,16384,4096 2048,8192,8192 8192,2048,8192 10240,8192,2048 16384,1024,16384 5120,5120,5120 \
  > $OUT/fp8_arms.jsonl 2> $OUT/fp8_arms.err || exit $?
echo done
