#!/bin/bash
# Round-2 pass L (experiment build, PDMB_EXPERIMENTS=1): W4S vs W4S with the per-round rotating
# XCD block map (x_w4s_rot): interleaved A/B and the per-XCD end times (tile timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PDMB_EXPERIMENTS=1 PDMB_NO_AUTOBUILD=1
OUT=gpurun_out/${1:-r2l}
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 100 --timeout-method thread -k "w4s" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tile_timeline.py --kernels w4s,x_w4s_rot --shapes 16384,16384,16384 8192,8192,8192 > $OUT/timeline.log 2>&1
rc=$?; tail -6 $OUT/timeline.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --rounds 7 --iters 10 --kernels w4s,x_w4s_rot,torch \
  --shapes 16384,16384,16384 8192,8192,8192 16384,16384,4096 > $OUT/ab.log 2>&1
rc=$?; tail -9 $OUT/ab.log; exit $rc
