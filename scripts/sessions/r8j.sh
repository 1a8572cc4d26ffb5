#!/bin/bash
# Round 6 session J (PDMB_EXPERIMENTS=1 build in the tree): does the fp8 W4S K4
# form also pay at 8-12 K-tiles (K = 1024 / 1536)? r8d / r8e measured +0.8 to
# +3.2 % there on three grids. More grids, settled, two sessions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8j; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels fp8_w4s,x_fp8_w4s_k4,torch \
  --shapes 16384,16384,1024 8192,8192,1024 16384,8192,1024 12288,12288,1024 4096,16384,1024 \
           16384,16384,1536 8192,8192,1536 6144,6144,1536 12288,12288,1536 \
  > $OUT/ab_fp8_k4_mid.jsonl 2> $OUT/ab_fp8_k4_mid.err || exit $?
grep '"summary"' $OUT/ab_fp8_k4_mid.jsonl | cut -c1-200
echo "exit 0"
