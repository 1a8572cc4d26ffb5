#!/bin/bash
# Round-2 GPU pass F: fp32 W4 (mid-tile barrier) exactness + A/B vs f32_256s and hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2f
mkdir -p $OUT
step() { local name=$1; shift; echo "== $name"; "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -12 $OUT/$name.log; echo "== $name rc=$rc"; return $rc; }
step f32_tests timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "f32 or fp32 or generic or thin" &&
step f32_ab timeout -k 10 300 python scripts/ab_kernels.py --kernels f32_256s,f32_w4 --dtype float32 --sizes 8192 16384 --rounds 4 --iters 5 &&
step f32_torch timeout -k 10 300 python scripts/gemm_perf.py --sizes 16384 --dtype float32 --rounds 3 --iters 5 --kernel f32_w4
