#!/bin/bash
# Round 6 session V (PDMB_EXPERIMENTS=1 build): the lean exact-fp32 tile arms
# (the W4 lean K-loop carried into f32_t128 / f32_t128x2 / f32_t64 / f32_t64x2:
# descriptors once per slice, K-tile offsets in the voffsets, M0 in one SALU,
# the DMA piece fused with its gap's MFMA) against their shipping kernels at
# the plan auto runs (same split), hipBLASLt last; settled, two sessions. The
# grids: matrix_parallel's fp32 shards at 4k / 8k and small grids whose auto
# plan is one of these kernels (split or not).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8v; mkdir -p $OUT
export PDMB_EXPERIMENTS=1
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench > $OUT/build.log 2>&1 || exit $?
timeout -k 10 300 python scripts/check_f32_tile_lean.py > $OUT/check_lean.jsonl 2> $OUT/check_lean.err || { tail -5 $OUT/check_lean.jsonl; tail -5 $OUT/check_lean.err; exit 1; }
tail -1 $OUT/check_lean.jsonl
ab() {  # name, kernels, shapes...
  local n=$1 k=$2; shift 2
  timeout -k 10 500 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 10 --settle 1 --sessions 2 \
    --kernels $k,torch --shapes "$@" > $OUT/ab_$n.jsonl 2> $OUT/ab_$n.err || return $?
  grep '"summary"' $OUT/ab_$n.jsonl | cut -c1-150
}
ab t128x2 f32_t128x2:1,x_f32_t128x2_lean:1 4096,2048,4096 8192,1024,8192 4096,4096,4096 3072,3072,2048 || exit $?
ab t128 f32_t128:1,x_f32_t128_lean:1 4096,1024,4096 2048,2048,2048 4096,2048,4096 || exit $?
ab t64 f32_t64:1,x_f32_t64_lean:1 4096,512,4096 2048,1024,2048 || exit $?
ab t64x2 f32_t64x2:2,x_f32_t64x2_lean:2 1536,3072,1024 2560,2048,4096 4608,4608,4096 || exit $?
echo "exit 0"
