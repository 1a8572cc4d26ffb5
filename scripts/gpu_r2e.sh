#!/bin/bash
# Round-2 GPU pass E: generic tile family (T128 / T128x2 / T256x128) exactness, then the
# interleaved sweep of every (kernel, split) arm vs hipBLASLt for the planner fit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2e
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -12 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step gemm_tests timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread &&
step sweep timeout -k 10 500 python scripts/splitk_sweep.py --rounds 4 --arms auto w4:1 w4:2 t256x128:1 t256x128:2 t128:1 t128:2 t128x2:1 --shapes 8192x1024x8192 4096x2048x4096 4096x1024x4096 4096x512x4096 2048x2048x2048 8192x2048x8192 16384x2048x16384 16384x16384x16384
