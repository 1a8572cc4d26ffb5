#!/bin/bash
# Round-2 GPU pass D: T128 ring depth A/B (4-stage 1 WG/CU vs 2-stage 2 WG/CU) on the shard shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2d
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -40 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step x2_exact timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "t128" &&
step sweep timeout -k 10 400 python scripts/splitk_sweep.py --rounds 4 --arms auto w4:2 t128:1 t128x2:1 t128:2 t128x2:2 --shapes 4096x2048x4096 8192x1024x8192 4096x1024x4096 2048x2048x2048 4096x512x4096 8192x2048x8192 16384x16384x16384
