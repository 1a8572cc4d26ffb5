#!/bin/bash
# round-5 session az: bf16 grids of 160 256^2 tiles (62.5 % of the CUs), the
# split arms of every tile (incl. 3-way below the 32-K-tile minimum), settled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; OUT=gpurun_out/r7az; mkdir -p $OUT
timeout -k 10 900 python scripts/ab_kernels.py --dtype bfloat16 --rounds 3 --iters 10 --settle 1 --sessions 1 \
  --kernels auto,torch,w4:2,w4:3,w4:4,t256x128:2,t256x128:3,t192x128:2,t192x128:3,t128:2,t128:3,t192:2,t192:3 \
  --shapes 2560,4096,4096 5120,2048,4096 2560,4096,8192 5120,2048,8192 4096,2560,4096 2048,5120,8192 \
  > $OUT/ab_bf16_160tile_arms.jsonl 2> $OUT/ab.err || exit $?
echo done
