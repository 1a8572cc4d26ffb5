#!/bin/bash
# Planner fit check: each tile kernel at its planned split vs auto vs hipBLASLt on the
# matrix_parallel shard shapes and edge shapes (profiles/r2_planner_fit.jsonl).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2kt}
mkdir -p $OUT
timeout -k 10 600 python -u scripts/ab_kernels.py --rounds 5 --iters 10 --kernels w4,t256x128,t128,t128x2,auto,torch \
  --shapes 4096,512,4096 4096,1024,4096 8192,1024,8192 8192,2048,8192 16384,2048,16384 4096,2048,4096 \
  3000,7000,5056 2000,3000,4096 6000,6000,6144 > $OUT/ab.log 2>&1
rc=$?; cut -c1-110 $OUT/ab.log | tail -60; exit $rc
