#!/bin/bash
# Round 6 session L (PDMB_EXPERIMENTS=1 build in the tree): exact fp32,
# x_f32_w4_nbp (the branch-free f32_w4 with 1024-B B rows, so its b128 B reads
# are conflict-free) against x_f32_w4_nb (first arm: bitwise column), the auto
# kernel (f32_t128x2) and hipBLASLt on the full grids, settled, two sessions;
# then the PMC passes with the instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8l; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== fp32 A/B $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float32 --rounds 3 --iters 5 --settle 1 --sessions 2 \
  --kernels x_f32_w4_nb,x_f32_w4_nbp,f32_t128x2,torch --shapes 16384,16384,16384 8192,8192,8192 4096,4096,4096 \
  > $OUT/ab_f32_nbp.jsonl 2> $OUT/ab_f32_nbp.err || exit $?
grep '"summary"' $OUT/ab_f32_nbp.jsonl | cut -c1-200
grep -h '"bitwise_eq_first"' $OUT/ab_f32_nbp.jsonl | grep x_f32_w4_nbp | cut -c1-220 | head -3
echo "== pmc $(date +%T)"
MIX=1 DT=float32 N=16384 KS=f32_t128x2,x_f32_w4_nb,x_f32_w4_nbp REPS=3 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle f32_t128x2,x_f32_w4_nb,x_f32_w4_nbp,torch
echo "exit 0"
