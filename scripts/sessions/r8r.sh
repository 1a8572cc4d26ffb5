#!/bin/bash
# Round 6 session R (PDMB_EXPERIMENTS=1 build in the tree): the streamed
# exact-fp32 W4 kernel (x_f32_w4s) and its non-streamed form (x_f32_w4_lean2)
# against the auto kernel and hipBLASLt on the whole-tile fp32 grids beyond the
# three squares: the matrix_parallel shards of 8k / 16k at ws = 2 / 4 / 8, more
# squares, long and short K. Settled, two sessions (first arm auto: the
# bitwise column shows where the plans already agree).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8r; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== fp32 grids A/B $(date +%T)"
timeout -k 10 1000 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 3 --settle 1 --sessions 2 \
  --kernels auto,x_f32_w4_lean2,x_f32_w4s,torch \
  --shapes 8192,4096,8192 8192,2048,8192 8192,1024,8192 16384,8192,16384 16384,4096,16384 16384,2048,16384 \
           6144,6144,6144 10240,10240,10240 12288,12288,12288 4096,4096,16384 16384,16384,1024 12288,6144,4096 \
  > $OUT/ab_f32_grids.jsonl 2> $OUT/ab_f32_grids.err || exit $?
grep '"summary"' $OUT/ab_f32_grids.jsonl | cut -c1-200
echo "exit 0"
