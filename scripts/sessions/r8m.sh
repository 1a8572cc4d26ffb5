#!/bin/bash
# Round 6 session M (PDMB_EXPERIMENTS=1 build in the tree): where does the
# branch-free exact-fp32 W4 kernel (x_f32_w4_nbp, 97.3 % MFMA busy) lose its
# last 1.4 % to hipBLASLt (98.7 %)? Timing-only variants (WRONG results) each
# drop one consumer: the DMA refills, the fragment reads, both (MFMAs + the
# mid-tile barrier), everything (MFMAs only). Settled A/B at 16k and 8k, then
# the PMC passes (MFMA busy, clock) at 16k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8m; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
KS=x_f32_w4_nbp,diag_f32_w4_nodma,diag_f32_w4_nofrag,diag_f32_w4_mfma_bar,diag_f32_w4_mfma_only,f32_t128x2
echo "== fp32 diag A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 1 \
  --kernels $KS,torch --shapes 16384,16384,16384 8192,8192,8192 \
  > $OUT/ab_f32_diag.jsonl 2> $OUT/ab_f32_diag.err || exit $?
grep '"summary"' $OUT/ab_f32_diag.jsonl | cut -c1-200
echo "== pmc $(date +%T)"
DT=float32 N=16384 KS=$KS REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle $KS,torch
echo "exit 0"
