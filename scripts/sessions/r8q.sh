#!/bin/bash
# Round 6 session Q (PDMB_EXPERIMENTS=1 build in the tree): the streamed
# persistent exact-fp32 W4 kernel (x_f32_w4s: lean2's K-loop as one K-tile
# stream per CU). First its exactness screen
# (scripts/check_f32_w4s.py: fp64 and bitwise against x_f32_w4_lean2), then the
# settled A/B against lean2 (first arm: bitwise column), the auto kernel
# (f32_t128x2) and hipBLASLt on the full grids, two sessions; then PMC at 16k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8q; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== exactness $(date +%T)"
timeout -k 10 300 python scripts/check_f32_w4s.py > $OUT/check.jsonl 2> $OUT/check.err || { cat $OUT/check.jsonl; tail -5 $OUT/check.err; exit 1; }
cat $OUT/check.jsonl
KS=x_f32_w4_lean2,x_f32_w4s,f32_t128x2
echo "== fp32 streamed A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels $KS,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_w4s.jsonl 2> $OUT/ab_f32_w4s.err || exit $?
grep '"summary"' $OUT/ab_f32_w4s.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_w4s.jsonl | grep -v summary | grep x_f32_w4s | cut -c1-220 | head -6
echo "== pmc $(date +%T)"
DT=float32 N=16384 KS=$KS REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle $KS,torch
echo "exit 0"
