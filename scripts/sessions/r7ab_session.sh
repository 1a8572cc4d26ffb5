#!/bin/bash
# round-5 session ab: the 192-row fp8 tiles forced on the 1-2-wave fp8 grids where auto (W4 / W4S) trails
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7ab; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 5 \
  --kernels auto,fp8_t192,fp8_t192x128,fp8_t256x128,torch \
  --shapes 5120,5120,5120 5120,5120,4096 4608,4608,3072 6144,4096,4096 10240,8192,2048 8192,2048,8192 4096,16384,4096 \
  > $OUT/ab_fp8_t192_midwave.jsonl 2> $OUT/ab.err || exit $?
echo done
