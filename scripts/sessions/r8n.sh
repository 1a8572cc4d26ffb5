#!/bin/bash
# Round 6 session N (PDMB_EXPERIMENTS=1 build in the tree): r8m found the
# branch-free exact-fp32 W4 kernel loses 0.9 % MFMA busy to its DMA refills and
# 0.6 % to its fragment reads, both issued in bursts (one per 4 MFMAs over a
# quarter of each half). x_f32_w4_spread* spread them over the half (DMA one
# per 16 MFMAs, reads one per 12): settled A/B against x_f32_w4_nbp (first arm:
# bitwise column), the auto kernel (f32_t128x2) and hipBLASLt, two sessions;
# then the PMC passes at 16k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8n; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
KS=x_f32_w4_nbp,x_f32_w4_spread,x_f32_w4_spread_dma,x_f32_w4_spread_rd,f32_t128x2
echo "== fp32 spread A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels $KS,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_spread.jsonl 2> $OUT/ab_f32_spread.err || exit $?
grep '"summary"' $OUT/ab_f32_spread.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_spread.jsonl | grep -v summary | grep spread | cut -c1-220 | head -9
echo "== pmc $(date +%T)"
DT=float32 N=16384 KS=$KS REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle $KS,torch
echo "exit 0"
