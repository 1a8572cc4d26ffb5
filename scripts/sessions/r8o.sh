#!/bin/bash
# Round 6 session O (PDMB_EXPERIMENTS=1 build in the tree): r8n found that
# spreading the DMA pieces and fragment reads over each half changes nothing:
# the cost is per instruction. x_f32_w4_lean cuts the K-loop's SALU from 72 to
# 29 per 512 MFMAs (descriptors built once per slice, the K-tile offset in the
# voffsets, M0 in one SALU). Settled A/B against x_f32_w4_nbp (first arm:
# bitwise column), the auto kernel (f32_t128x2) and hipBLASLt, two sessions;
# then the PMC passes at 16k with the instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8o; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
KS=x_f32_w4_nbp,x_f32_w4_lean,f32_t128x2
echo "== fp32 lean A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels $KS,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_lean.jsonl 2> $OUT/ab_f32_lean.err || exit $?
grep '"summary"' $OUT/ab_f32_lean.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_lean.jsonl | grep -v summary | grep lean | cut -c1-220 | head -9
echo "== pmc $(date +%T)"
MIX=1 DT=float32 N=16384 KS=$KS REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle $KS,torch
echo "exit 0"
