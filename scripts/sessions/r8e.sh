#!/bin/bash
# Round 6 session E (PDMB_EXPERIMENTS=1 build in the tree): the fp8 W4S K4 form
# (first-pair DMA targets through selects; also runs K = 512) against the
# shipping fp8 W4S on the long-K grids where W4S ships today, settled, two
# sessions; then its bitwise tests against fp8 W4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PDMB_EXPERIMENTS=1
OUT=gpurun_out/r8e; mkdir -p $OUT
timeout -k 10 900 python -m pytorch_distributed_matmul_benchmark_amd.ops.build --no-bench -v > $OUT/build.log 2>&1 || exit $?
echo "== k4 tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -m "gpu and experiments" -k k4 -x -q \
  --timeout 120 --timeout-method thread > $OUT/k4_tests.log 2>&1 || { tail -20 $OUT/k4_tests.log; exit 1; }
tail -2 $OUT/k4_tests.log
echo "== long K $(date +%T)"
timeout -k 10 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --rounds 4 --iters 10 --settle 1 --sessions 2 \
  --kernels fp8_w4s,x_fp8_w4s_k4,torch \
  --shapes 16384,16384,16384 8192,8192,8192 16384,2048,16384 16384,4096,16384 8192,4096,8192 \
           16384,16384,2048 16384,16384,4096 8192,8192,2048 6144,6144,1536 \
  > $OUT/ab_fp8_w4s_vs_k4.jsonl 2> $OUT/ab_fp8_w4s_vs_k4.err || exit $?
grep '"summary"' $OUT/ab_fp8_w4s_vs_k4.jsonl | cut -c1-200
echo "exit 0"
