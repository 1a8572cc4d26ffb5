#!/bin/bash
# Round 6 session U: f32_w4s with its outstanding-VMEM bound (<= 63 at every
# point: K-tile 0 waits vmcnt(47), the epilogue vmcnt(43) before its last 20
# stores, no stand-in loads; tests/test_vmcnt_bound.py). Shipping build:
# cold first launches, one per fresh process, under short timeouts; the fp32
# GPU tests; the exact-integer race screen; the fp32 table. Then the
# PDMB_EXPERIMENTS=1 build: the lean exact-fp32 tile arms' exactness screen.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r8u; mkdir -p $OUT
for s in "256 256 128" "4096 4096 256" "4096 4096 4096" "8192 8192 512" "1024 1024 512 3" "16384 16384 256" \
         "256 256 128" "2304 8960 384"; do
  timeout -k 5 45 python scripts/w4s_probe.py $s >> $OUT/probe_ship.jsonl 2>> $OUT/probe_ship.err || { echo "ship $s rc=$?"; cat $OUT/probe_ship.jsonl; exit 1; }
done
cat $OUT/probe_ship.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "f32" > $OUT/pytest_f32.log 2>&1 || { tail -30 $OUT/pytest_f32.log; exit 1; }
tail -2 $OUT/pytest_f32.log
timeout -k 10 300 python scripts/race_screen.py --reps 50 --kernels f32_w4s > $OUT/race_f32_w4s.jsonl 2>&1 || exit $?
cut -c1-150 $OUT/race_f32_w4s.jsonl
timeout -k 10 400 python scripts/ab_kernels.py --dtype float32 --rounds 4 --iters 5 --settle 1 --sessions 2 \
  --kernels auto,f32_t128x2,torch --sizes 4096 8192 16384 > $OUT/table_float32.jsonl 2> $OUT/table_float32.err || exit $?
grep '"summary"' $OUT/table_float32.jsonl | cut -c1-160
PDMB_EXPERIMENTS=1 timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench > $OUT/build.log 2>&1 || exit $?
timeout -k 10 300 python scripts/check_f32_tile_lean.py > $OUT/check_lean.jsonl 2> $OUT/check_lean.err || { tail -5 $OUT/check_lean.jsonl; tail -5 $OUT/check_lean.err; exit 1; }
tail -1 $OUT/check_lean.jsonl
echo "exit 0"
