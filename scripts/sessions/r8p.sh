#!/bin/bash
# Round 6 session P (PDMB_EXPERIMENTS=1 build in the tree): r8o's lean
# exact-fp32 W4 (29 SALU per 512 MFMAs instead of 72) gained 0.5-0.8 % and tied
# the auto kernel. x_f32_w4_lean2 also drops the s_nop of each of the 16 DMA
# pieces (the piece's M0 write and load wrap its gap's MFMA in one asm block).
# Settled A/B against x_f32_w4_lean (first arm: bitwise column), f32_t128x2 and
# hipBLASLt, two sessions; then the PMC passes at 16k with the instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8p; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
KS=x_f32_w4_lean,x_f32_w4_lean2,f32_t128x2
echo "== fp32 lean A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels $KS,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_lean2.jsonl 2> $OUT/ab_f32_lean2.err || exit $?
grep '"summary"' $OUT/ab_f32_lean2.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_lean2.jsonl | grep -v summary | grep lean2 | cut -c1-220 | head -9
echo "== pmc $(date +%T)"
MIX=1 DT=float32 N=16384 KS=$KS REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle $KS,torch
echo "exit 0"
