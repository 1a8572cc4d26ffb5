#!/bin/bash
# Round 6 session I (PDMB_EXPERIMENTS=1 build in the tree): exact fp32, the
# branch-free K-loop of f32_w4 (x_f32_w4_nb: 0 branches per 512 MFMAs instead of
# 32) against f32_w4, the auto kernel (f32_t128x2) and hipBLASLt on the full
# grids, settled, two sessions (first arm f32_w4: bitwise column); then the
# PMC passes with the instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8i; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== fp32 A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels f32_w4,x_f32_w4_nb,f32_t128x2,auto,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_nb.jsonl 2> $OUT/ab_f32_nb.err || exit $?
grep '"summary"' $OUT/ab_f32_nb.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_nb.jsonl | grep x_f32_w4_nb | cut -c1-220 | head -3
echo "== pmc $(date +%T)"
MIX=1 DT=float32 N=16384 KS=f32_t128x2,f32_w4,x_f32_w4_nb REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle f32_t128x2,f32_w4,x_f32_w4_nb,torch
echo "exit 0"
