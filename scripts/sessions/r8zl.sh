#!/bin/bash
# Round 6 session ZL (PDMB_EXPERIMENTS=1 build, built on the box): PMC passes on
# fp8 4096 x 16384 x 1024, the worst mid-K fp8 grid (0.90 of hipBLASLt):
# shipping W4S, the thin 4 x 64 round (+3.4 %, r8zj) and hipBLASLt. Where do the
# other 7 points go: MFMA busy, L2 hit rate, read requests?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8zl; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench > $OUT/build.log 2>&1 || exit $?
KS=fp8_w4s,x_fp8_w4s_thin DT=float8_e4m3fn SHAPE=4096,16384,1024 REPS=20 OUT=$OUT/pmc \
  timeout -k 10 900 bash scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT/pmc --cycle fp8_w4s,x_fp8_w4s_thin,torch > $OUT/summary.txt 2>&1
tail -14 $OUT/summary.txt
echo "exit 0"
