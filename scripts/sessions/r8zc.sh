#!/bin/bash
# Round 6 session ZC (PDMB_EXPERIMENTS=1 build): the lean W4S arm
# (x_w4s_lean: the tile's descriptors at K = 0, K-tile offsets in the
# voffsets, DMA pieces fused with their gap's MFMA outside the first two
# K-tiles; 188 instead of 260 non-MFMA instructions per 256 MFMAs). Exactness
# screen, then settled A/B against the shipping W4S and hipBLASLt, bf16, two
# sessions; then a PMC pass at 16k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8zc; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench > $OUT/build.log 2>&1 || exit $?
timeout -k 10 300 python scripts/check_w4s_lean.py > $OUT/check.jsonl 2> $OUT/check.err || { tail -5 $OUT/check.jsonl; tail -5 $OUT/check.err; exit 1; }
tail -1 $OUT/check.jsonl
timeout -k 10 700 python scripts/ab_kernels.py --dtype bfloat16 --rounds 4 --iters 20 --settle 1 --sessions 2 \
  --kernels w4s,x_w4s_lean,torch --shapes 16384,16384,16384 8192,8192,8192 16384,2048,16384 8192,4096,8192 \
  4096,4096,4096,4 16384,16384,2048 > $OUT/ab_lean.jsonl 2> $OUT/ab_lean.err || exit $?
grep '"summary"' $OUT/ab_lean.jsonl | cut -c1-170
KS=w4s,x_w4s_lean DT=bfloat16 N=16384 REPS=3 OUT=$OUT/pmc timeout -k 10 600 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle w4s,x_w4s_lean,torch 2>&1 | tail -12
echo "exit 0"
