#!/bin/bash
# round-5 session bb: fp8 short-K grids (4-8 K-tiles), every fp8 kernel arm
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7bb; mkdir -p $OUT
timeout -k 10 600 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 3 --iters 20 --settle 1 --sessions 1 \
  --kernels auto,torch,fp8_w4,fp8_w4s,fp8_t256x128,fp8_t128,fp8_t192,fp8_t192x128 \
  --shapes 16384,16384,512 16384,16384,1024 8192,4096,1024 8192,8192,512 16384,8192,512 \
  > $OUT/ab_fp8_short_k_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
